# round 5: decode kernel in 4-wave workgroups (two per CU: one's start-up beside the other's tiles) (nw4)
set -o pipefail
O=$PWD/gpurun_out/r05ac
mkdir -p $O
L=$PWD/variants/var_nw4/libwakeword.so
WAKEWORD_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_ctc.py tests/test_gpu_configs.py -m gpu -q -s --timeout 300 --timeout-method thread -k "ctc or config5" > $O/tests.log 2>&1; rc=$?
[ $rc -le 1 ] || { tail -20 $O/tests.log; exit $rc; }
tail -2 $O/tests.log; grep "config5 decisions" $O/tests.log | grep -v print | cut -c1-120
bash tools/debug/ctc_ab.sh nw4 2>&1 | tee $O/ab.txt
