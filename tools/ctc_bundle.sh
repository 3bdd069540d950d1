#!/bin/bash
# Config-5 (CTC head) measurement bundle, run on the GPU box through gpurun:
#   bash tools/ctc_bundle.sh <tag>  ->  gpurun_out/ctc_<tag>/{ctc,ctc_fp32}.log + rocprofv3 kernel stats
# then, in the build container: bash tools/ctc_bundle.sh <tag> --collect  (copies into profiles/)
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
T=${1:?tag}
O=$R/gpurun_out/ctc_$T
if [ "$2" = "--collect" ]; then
  grep '^{' "$O/ctc.log" | tail -1 > "$R/profiles/${T}_ctc.json"
  grep '^{' "$O/ctc_fp32.log" | tail -1 > "$R/profiles/${T}_ctc_fp32.json"
  cp "$O/trace/run_kernel_stats.csv" "$R/profiles/${T}_ctc_kernel_stats.csv"
  exit 0
fi
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python bench_ctc.py > "$O/ctc.log" 2>&1 || exit $?
timeout -k 10 300 python bench_ctc.py --precision fp32 > "$O/ctc_fp32.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
  python3 "$R/bench_ctc.py" > "$O/prof.log" 2>&1 || exit $?
for f in ctc ctc_fp32; do echo "$f: $(grep '^{' $O/$f.log | tail -1 | cut -c1-300)"; done
