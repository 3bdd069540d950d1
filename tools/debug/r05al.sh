# round 5, K = 32 question: the fused kernel's front-end role alone
# (WAKEWORD_FUSED_EXP=1) with the CNN waves replaced by a bare register-operand
# MFMA stream (-DWK_DIAG_K32_SPIN: 1 = K = 32 bf16, 0 = K = 16 pair).
# Power-row snapshot A across launches (tools/debug/prow_probe.py).
set -o pipefail
O=$PWD/gpurun_out/r05al
mkdir -p $O
for v in spin16 spin32; do
  echo "== $v" >> $O/spin.txt
  WAKEWORD_FUSED_EXP=1 WAKEWORD_LIB=$PWD/variants/var_$v/libwakeword.so timeout -k 10 240 python tools/debug/prow_probe.py bf16 4 >> $O/spin.txt 2>&1 || { cat $O/spin.txt; exit 1; }
done
grep -v amdgpu.ids $O/spin.txt
