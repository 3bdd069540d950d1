#!/bin/bash
# One GPU round trip for a code change (run through gpurun): the -m gpu parity
# suite, then the default bench line (fp32), the bf16 line, and bench.py's
# self-launched 2-rank path rehearsed on one GPU over gloo.
#   bash tools/gpu_check.sh [tag]     -> gpurun_out/check_<tag>/
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
T=${1:-x}
O=$R/gpurun_out/check_$T
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gputest.log" 2>&1
rc=$?; tail -3 "$O/gputest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python bench.py --no-cpu-baseline > "$O/bench_fp32.log" 2>&1 || exit $?
timeout -k 10 180 python bench.py --no-cpu-baseline --precision bf16 > "$O/bench_bf16.log" 2>&1 || exit $?
timeout -k 10 240 python bench.py --no-cpu-baseline --gpus 2 --dist-backend gloo > "$O/bench_gloo2.log" 2>&1 || exit $?
for f in fp32 bf16 gloo2; do python -c "import json,sys;d=json.loads(open('$O/bench_$f.log').read().strip().splitlines()[-1]);print('$f', d['n_gpus'], 'rehearsal' if d.get('rehearsal') else (round(d['value']/1e6,3),'M win/s', d['roofline']['launch_ms'],'ms frac',d['roofline']['frac']), d['config'].get('process_group_world_size'))"; done
