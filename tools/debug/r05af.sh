# round 5: encoder inside GRU layer 0 (genc): CTC tests on it, then A/B + kernel stats
set -o pipefail
O=$PWD/gpurun_out/r05af
mkdir -p $O
L=$PWD/variants/var_genc/libwakeword.so
WAKEWORD_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_ctc.py tests/test_gpu_configs.py -m gpu -v -s --timeout 300 --timeout-method thread -k "ctc or config5" > $O/tests.log 2>&1; rc=$?
[ $rc -le 1 ] || { tail -30 $O/tests.log; exit $rc; }
tail -3 $O/tests.log; grep "config5 decisions\|FAILED" $O/tests.log | grep -v print | cut -c1-140
bash tools/debug/ctc_ab.sh genc 2>&1 | tee $O/ab.txt
