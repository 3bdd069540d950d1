#!/bin/bash
# HBM traffic of the config-5 stages (run on the GPU box through gpurun):
# two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over bench_ctc.py, then
# tools/ctc_traffic.py maps the kernels to bench_ctc's stages.
#   bash tools/ctc_traffic.sh <tag>  ->  gpurun_out/ctctraffic_<tag>/{pmc.json,ctc_hbm_traffic.json}
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
T=${1:?tag}
O=$R/gpurun_out/ctctraffic_$T
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d "$O/p$i" -o run --output-format csv -- python3 "$R/bench_ctc.py" \
    --steps 2 --warmup 1 --no-cpu-baseline > "$O/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$O/p$i.log"; exit 1; }
done
cd "$R"
python tools/pmc_summary.py "$O" --json "$O/pmc.json" > "$O/pmc_summary.txt" || exit $?
python tools/ctc_traffic.py "$O/pmc.json" "profiles/${T}_ctc_pmc_traffic.json" > "$O/ctc_hbm_traffic.json" || exit $?
cat "$O/ctc_hbm_traffic.json"
