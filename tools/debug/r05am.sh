# round 5, K = 32 question: front-end register dumps at four points of fe_rest,
# front-end role alone + bare MFMA stream (fd16: K = 16 pair, fd32: K = 32 bf16)
set -o pipefail
O=$PWD/gpurun_out/r05am
mkdir -p $O
for v in fd16 fd32; do
  echo "== $v" >> $O/fedump.txt
  WAKEWORD_FUSED_EXP=1 WK_PROW_CLIPS=4 WAKEWORD_LIB=$PWD/variants/var_$v/libwakeword.so timeout -k 10 300 python tools/debug/fe_dump_probe.py bf16 4 >> $O/fedump.txt 2>&1 || { cat $O/fedump.txt; exit 1; }
done
grep -v amdgpu.ids $O/fedump.txt
