set -o pipefail
O=$PWD/gpurun_out/r04r
mkdir -p $O
for v in spin2 spin3; do
  WAKEWORD_LIB=$PWD/variants/var_$v/libwakeword.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_protocol.py tests/test_gpu_bf16.py -q -x --timeout 120 --timeout-method thread > $O/test_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 $O/test_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/debug/ab.sh prod spin2 spin3 prod spin2 spin3 2>&1 | tee $O/ab.txt
