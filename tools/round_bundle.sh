#!/bin/bash
# Everything the round's docs quote, in one GPU call (run through gpurun):
#   bash tools/round_bundle.sh <tag>
# profile bundles of the headline (fp32) and config 4 (bf16) lines
# (tools/profile_round.sh: bench + rocprofv3 kernel stats + PMC + HBM traffic),
# then the streaming (config 3), CTC (config 5) and call-surface benches.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
T=${1:?tag}
cd "$R"
bash tools/profile_round.sh "${T}" || exit $?
bash tools/profile_round.sh "${T}_bf16" --precision bf16 || exit $?
O=$R/gpurun_out/extra_$T
mkdir -p "$O"
timeout -k 10 300 python bench_stream.py > "$O/stream.log" 2>&1 || exit $?
timeout -k 10 300 python bench_ctc.py > "$O/ctc.log" 2>&1 || exit $?
timeout -k 10 300 python bench_ctc.py --precision fp32 > "$O/ctc_fp32.log" 2>&1 || exit $?
timeout -k 10 300 python bench_surfaces.py > "$O/surfaces.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --precision bf16x3 > "$O/bench_bf16x3.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ctc_trace" -o run -- \
  python3 "$R/bench_ctc.py" > "$O/ctc_prof.log" 2>&1 || exit $?
for f in stream ctc ctc_fp32 surfaces bench_bf16x3; do echo "$f: $(grep '^{' $O/$f.log | tail -1 | cut -c1-300)"; done
