#!/bin/bash
# Issue-level PMC (tools/debug/groups_issue.txt) of the fused kernel per role:
# CONFIGS="prec:exp ..." (exp 0 = fused, 1 = front-end role alone, 2 = CNN role
# alone; needs the -DWK_DIAG variant build/var_exp).
export WAKEWORD_LIB=$PWD/esp32-wake-word_amd/build/var_exp/libwakeword.so
for cfg in ${CONFIGS:-fp32:0 fp32:1 fp32:2 bf16:0}; do
  p=${cfg%%:*}; x=${cfg##*:}
  WAKEWORD_FUSED_EXP=$x bash tools/debug/pmc_groups.sh gpurun_out/pmc_${p}_${x} tools/debug/groups_issue.txt \
    --steps 2 --warmup 1 --no-cpu-baseline --precision $p || exit 1
done
