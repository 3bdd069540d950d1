set -o pipefail
O=$PWD/gpurun_out/r04o
mkdir -p $O
WAKEWORD_LIB=$PWD/variants/var_pw2/libwakeword.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x --timeout 120 --timeout-method thread > $O/test_pw2.log 2>&1; rc=$?; tail -2 $O/test_pw2.log; [ $rc -eq 0 ] || exit $rc
bash tools/debug/ab.sh prod pw2 prod pw2 2>&1 | tee $O/ab.txt
