# round 5: decode kernel with one wave per SIMD (4 waves, 96 / 64 rows each), y fragments in AGPRs (r6a, r4a)
set -o pipefail
O=$PWD/gpurun_out/r05z
mkdir -p $O
WAKEWORD_LIB=$PWD/variants/var_r6a/libwakeword.so timeout -k 10 600 python -u -m pytest tests/test_ctc.py tests/test_gpu_configs.py -m gpu -q -s --timeout 300 --timeout-method thread -k "ctc or config5" > $O/tests.log 2>&1; rc=$?
[ $rc -le 1 ] || { tail -20 $O/tests.log; exit $rc; }
tail -2 $O/tests.log; grep "config5 decisions" $O/tests.log | grep -v print | cut -c1-110
bash tools/debug/ctc_ab.sh r6a r4a 2>&1 | tee $O/ab.txt
