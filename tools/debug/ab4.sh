#!/bin/bash
# Four alternating passes of ab.sh's timing (fp32 and bf16) for a small expected difference.
#   [PRECS="fp32 bf16"] [PASSES=4] bash tools/debug/ab4.sh name1 name2 ...
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
for prec in ${PRECS:-fp32 bf16}; do
  for pass in $(seq ${PASSES:-4}); do
    for v in "$@"; do
      if [ "$v" = prod ]; then L=$R/esp32-wake-word_amd/wakeword/libwakeword.so; else L=$R/variants/var_$v/libwakeword.so; fi
      WAKEWORD_LIB=$L timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --precision $prec > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
      python -c "import json;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print('$prec $v', round(d['value']/1e6,3), 'M win/s', d['roofline']['launch_ms'])"
    done
  done
done
