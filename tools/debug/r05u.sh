# round 5: log-mel window pairs (lmwin2), decode-kernel runner-up carry (carry), both: CTC tests on both, then A/B
set -o pipefail
O=$PWD/gpurun_out/r05u
mkdir -p $O
WAKEWORD_LIB=$PWD/variants/var_both/libwakeword.so timeout -k 10 600 python -u -m pytest tests/test_ctc.py tests/test_gpu_configs.py -m gpu -v -s --timeout 300 --timeout-method thread -k "ctc or config5" > $O/tests.log 2>&1; rc=$?
[ $rc -le 1 ] || { tail -20 $O/tests.log; exit $rc; }
tail -3 $O/tests.log; grep "config5 decisions" $O/tests.log | grep -v print
bash tools/debug/ctc_ab.sh lmwin2 carry both 2>&1 | tee $O/ab.txt
