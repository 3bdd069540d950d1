# round 5, K = 32 question: the fused kernel's K = 32 build with the DFT16
# quarter turn as one packed op (-DWK_QTURN_PK); features repeatability, bf16
set -o pipefail
O=$PWD/gpurun_out/r05ap
mkdir -p $O
for v in k32q; do
  echo "== $v" >> $O/k32.txt
  WAKEWORD_LIB=$PWD/variants/var_$v/libwakeword.so timeout -k 10 240 python tools/debug/k32_repeat.py bf16 6 feats >> $O/k32.txt 2>&1 || { cat $O/k32.txt; exit 1; }
done
grep -v amdgpu.ids $O/k32.txt
