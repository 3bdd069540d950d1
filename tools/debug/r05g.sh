# round 5: log-mel wave ranges (lmr) + encoder grid / 8-wave variants: CTC tests on lmr, then A/B
set -o pipefail
O=$PWD/gpurun_out/r05g
mkdir -p $O
L=$PWD/variants/var_lmr/libwakeword.so
WAKEWORD_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_ctc.py tests/test_gpu_configs.py -m gpu -v -s --timeout 300 --timeout-method thread -k "ctc or config5" > $O/tests.log 2>&1; rc=$?
[ $rc -le 1 ] || { tail -20 $O/tests.log; exit $rc; }
tail -3 $O/tests.log; grep "config5 decisions" $O/tests.log
bash tools/debug/ctc_ab.sh lmr enc4 enc6 w8 w8win 2>&1 | tee $O/ab.txt
