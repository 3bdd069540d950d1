set -o pipefail
O=$PWD/gpurun_out/r04t
mkdir -p $O
WAKEWORD_LIB=$PWD/variants/var_wino/libwakeword.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_protocol.py -q -x --timeout 120 --timeout-method thread > $O/test_wino.log 2>&1; rc=$?; echo "wino: $(tail -1 $O/test_wino.log)"; [ $rc -eq 0 ] || exit $rc
bash tools/debug/ab.sh prod wino prod wino prod wino 2>&1 | tee $O/ab.txt
