#!/bin/bash
# Config-5 PMC bundle (run on the GPU box through gpurun): the counter passes
# of tools/profile_pmc.sh over bench_ctc.py, their per-kernel summary, and the
# per-stage HBM traffic (2 x FETCH_SIZE + WRITE_SIZE) that bench_ctc.py reads
# from profiles/ctc_hbm_traffic.json.
#   bash tools/ctc_pmc.sh <tag>   ->  gpurun_out/ctcpmc_<tag>/{pmc_summary.txt,pmc.json,ctc_hbm_traffic.json}
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
T=${1:?tag}
O=$R/gpurun_out/ctcpmc_$T
PMC_BENCH=bench_ctc.py bash "$R/tools/profile_pmc.sh" "$O" --steps 2 --warmup 1 --no-cpu-baseline || exit $?
cd "$R"
python tools/pmc_summary.py "$O" --json "$O/pmc.json" > "$O/pmc_summary.txt" || exit $?
python tools/ctc_traffic.py "$O/pmc.json" "profiles/${T}_ctc_pmc_summary.txt" > "$O/ctc_hbm_traffic.json" || exit $?
cat "$O/ctc_hbm_traffic.json"
