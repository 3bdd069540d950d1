#!/bin/bash
# fp32 vs int16 audio storage, two passes each (bench default config otherwise).
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
for a in f32 i16 f32 i16; do
  timeout -k 10 100 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --audio $a ${AUD_ARGS:-} > gpurun_out/aud_$a.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/aud_$a.log').read().strip().splitlines()[-1]);print('$a', round(d['value']/1e6,3))"
done
