# round 5, K = 32 question: roles split by hardware SIMD (front-end on SIMDs 0-1, CNN on 2-3).
# k16split: parity tests (the remap is correct) + repeatability; k32split vs k32: repeatability.
set -o pipefail
O=$PWD/gpurun_out/r05s
mkdir -p $O
WAKEWORD_LIB=$PWD/variants/var_k16split/libwakeword.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/k16split_parity.log 2>&1 || { tail -20 $O/k16split_parity.log; exit 1; }
tail -2 $O/k16split_parity.log
for v in k16split k32split k32; do
  echo "== $v" >> $O/k32.txt
  WAKEWORD_LIB=$PWD/variants/var_$v/libwakeword.so timeout -k 10 240 python tools/debug/k32_repeat.py bf16 6 >> $O/k32.txt 2>&1 || { cat $O/k32.txt; exit 1; }
done
grep -v amdgpu.ids $O/k32.txt
