#!/bin/bash
# rocprofv3 kernel stats of the config-5 bench (fp16).
R=$(cd "$(dirname "$0")/../.." && pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ctcprof" -o run -- python3 "$R/bench_ctc.py" --steps 3 ${CTC_ARGS:-} > "$R/gpurun_out/ctcprof.log" 2>&1 || exit 1
f=$(find "$R/gpurun_out/ctcprof" -name "run_kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | cut -c1-160
