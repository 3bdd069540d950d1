# round 5: decode-only output kernel with the fold interleaved among the MFMAs (dec32: 32x32x16): CTC tests, then A/B
set -o pipefail
O=$PWD/gpurun_out/r05y
mkdir -p $O
cp gpurun_out/r05m/ab.txt $O/probe_ab.txt 2>/dev/null
L=$PWD/variants/var_dec32/libwakeword.so
WAKEWORD_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_ctc.py tests/test_gpu_configs.py -m gpu -v -s --timeout 300 --timeout-method thread -k "ctc or config5" > $O/tests.log 2>&1; rc=$?
[ $rc -le 1 ] || { tail -20 $O/tests.log; exit $rc; }
tail -3 $O/tests.log; grep "config5 decisions" $O/tests.log | grep -v print
bash tools/debug/ctc_ab.sh dec32 2>&1 | tee $O/ab.txt
