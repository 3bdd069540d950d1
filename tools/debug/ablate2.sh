#!/bin/bash
# FE-alone (exp 1) and fused timing of ablation variants: bash tools/debug/ablate2.sh v1 v2 ...
# WAKEWORD_FUSED_EXP is honoured only by libraries built with -DWK_DEBUG_EXPERIMENTS
# (bash tools/debug/build_variant.sh exp -DWK_DEBUG_EXPERIMENTS; WAKEWORD_LIB=...var_exp/libwakeword.so).
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
for v in "$@"; do
  L=esp32-wake-word_amd/build/var_$v/libwakeword.so
  for x in 1 0; do
    WAKEWORD_LIB=$L WAKEWORD_FUSED_EXP=$x timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${ABL_ARGS:-} > gpurun_out/abl_${v}_$x.log 2>&1 || { echo "$v failed"; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/abl_${v}_$x.log').read().strip().splitlines()[-1]);print('$v exp=$x', round(d['roofline']['launch_ms'],4), 'ms')"
  done
done
