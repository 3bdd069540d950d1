#!/bin/bash
# Role isolation of the fused kernel (timing only; logits are wrong):
# WAKEWORD_FUSED_EXP is honoured only by libraries built with -DWK_DIAG
# (bash tools/debug/build_variant.sh exp -DWK_DIAG; WAKEWORD_LIB=...var_exp/libwakeword.so).
# for each precision, FE role alone (exp 1), CNN role alone (exp 2), both (0).
# PRECS / AUDIO select the precisions and the sample type (f32 / i16).
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
for p in ${PRECS:-fp32 bf16 bf16x3}; do
  for x in ${EXPS:-0 1 2}; do
    WAKEWORD_FUSED_EXP=$x timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --precision $p \
      --audio ${AUDIO:-f32} > gpurun_out/roles_${p}_${x}.log 2>&1 || { echo "$p $x failed"; tail -5 gpurun_out/roles_${p}_${x}.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/roles_${p}_${x}.log').read().strip().splitlines()[-1]);print('$p ${AUDIO:-f32} exp=$x', round(d['roofline']['launch_ms'],4), 'ms', round(d['value']/1e6,3), 'M win/s')"
  done
done
