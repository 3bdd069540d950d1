# round 5, K = 32 question: is the co-residence corruption specific to the bf16
# K = 32 MFMA, or shared by the f16 K = 32 form?  Repeatability of the features
# (the front-end's output; the f16 variant's logits are wrong by construction).
set -o pipefail
O=$PWD/gpurun_out/r05ag
mkdir -p $O
for v in prod k32 k32h; do
  if [ $v = prod ]; then L=""; else L="WAKEWORD_LIB=$PWD/variants/var_$v/libwakeword.so"; fi
  echo "== $v" >> $O/k32.txt
  env $L timeout -k 10 240 python tools/debug/k32_repeat.py bf16 6 feats >> $O/k32.txt 2>&1 || { cat $O/k32.txt; exit 1; }
done
grep -v amdgpu.ids $O/k32.txt
