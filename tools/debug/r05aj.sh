# round 5, K = 32 question: which conv layer's K = 32 MFMAs change the front-end
# (WK_K32_MASK: bit 0 conv1, 1 conv2, 2 conv3); features repeatability, bf16
set -o pipefail
O=$PWD/gpurun_out/r05aj
mkdir -p $O
for v in k32m1 k32m2 k32m4; do
  echo "== $v" >> $O/k32.txt
  WAKEWORD_LIB=$PWD/variants/var_$v/libwakeword.so timeout -k 10 240 python tools/debug/k32_repeat.py bf16 6 feats >> $O/k32.txt 2>&1 || { cat $O/k32.txt; exit 1; }
done
grep -v amdgpu.ids $O/k32.txt
