# round 5: encoder blocks of 16 utterances at one frame (enctm): CTC tests on it, then A/B
set -o pipefail
O=$PWD/gpurun_out/r05j
mkdir -p $O
L=$PWD/variants/var_enctm/libwakeword.so
WAKEWORD_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_ctc.py tests/test_gpu_configs.py -m gpu -v -s --timeout 300 --timeout-method thread -k "ctc or config5" > $O/tests.log 2>&1; rc=$?
[ $rc -le 1 ] || { tail -20 $O/tests.log; exit $rc; }
tail -3 $O/tests.log; grep "config5 decisions" $O/tests.log | grep -v print
bash tools/debug/ctc_ab.sh enctm 2>&1 | tee $O/ab.txt
