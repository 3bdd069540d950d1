#!/bin/bash
# Front-end role alone (WAKEWORD_FUSED_EXP=1) with 8 vs 12 front-end waves per workgroup
# (variants/var_diag8: -DWK_DIAG; var_diag12: -DWK_DIAG -DWK_FE_WAVES=12), alternating passes.
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
for pass in 1 2 3; do
  for v in diag8 diag12; do
    for p in ${PRECS:-fp32 bf16}; do
      WAKEWORD_LIB=$R/variants/var_$v/libwakeword.so WAKEWORD_FUSED_EXP=1 timeout -k 10 120 python bench.py --steps 10 --warmup 2 \
        --no-cpu-baseline --no-extras --precision $p > gpurun_out/few_${v}_$p.log 2>&1 || { echo "$v $p failed"; tail -5 gpurun_out/few_${v}_$p.log; exit 1; }
      python -c "import json;d=json.loads(open('gpurun_out/few_${v}_$p.log').read().strip().splitlines()[-1]);print('$v $p FE alone', round(d['roofline']['launch_ms'],4), 'ms')"
    done
  done
done
