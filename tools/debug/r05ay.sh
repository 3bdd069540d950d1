# round 5, K = 32 question: the K = 32 form beside the scalar-fp32 front-end
# (-DWK_FE_SCALAR: no packed fp32 in the fused kernel); features repeatability
set -o pipefail
O=$PWD/gpurun_out/r05ay
mkdir -p $O
for p in bf16 bf16x3; do
  WAKEWORD_LIB=$PWD/variants/var_k32s/libwakeword.so timeout -k 10 240 python tools/debug/k32_repeat.py $p 6 feats >> $O/k32.txt 2>&1 || { cat $O/k32.txt; exit 1; }
done
grep -v amdgpu.ids $O/k32.txt
