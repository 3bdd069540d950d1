set -o pipefail
O=$PWD/gpurun_out/r05e
mkdir -p $O
for v in k32 k32bperm k32dpppad k16bperm; do
  WAKEWORD_LIB=$PWD/variants/var_$v/libwakeword.so timeout -k 10 240 python tools/debug/k32_repeat.py bf16 6 >> $O/k32.txt 2>&1 || { cat $O/k32.txt; exit 1; }
done
for v in k32bperm; do
  WAKEWORD_LIB=$PWD/variants/var_$v/libwakeword.so timeout -k 10 240 python tools/debug/k32_repeat.py bf16x3 6 >> $O/k32.txt 2>&1 || { cat $O/k32.txt; exit 1; }
done
grep -v amdgpu.ids $O/k32.txt
