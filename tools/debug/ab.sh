#!/bin/bash
# A/B timing of library variants on the GPU box:  bash tools/debug/ab.sh name1 name2 ...
# (variants from build_variant.sh; "prod" = the in-tree library).  Two passes each.
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
for pass in 1 2; do
  for v in "$@"; do
    if [ "$v" = prod ]; then L=$R/esp32-wake-word_amd/wakeword/libwakeword.so; else L=$R/variants/var_$v/libwakeword.so; fi
    WAKEWORD_LIB=$L timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $AB_ARGS > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
    python -c "import json,sys;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print('$v', round(d['value']/1e6,3), 'M win/s', d['roofline']['frac'])"
  done
done
