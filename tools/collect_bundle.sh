#!/bin/bash
# Copy a round6_bundle.sh run's judged files from gpurun_out/ into profiles/.
#   bash tools/collect_bundle.sh <tag>
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=${1:?tag}
G=$R/gpurun_out P=$R/profiles
last_json() { grep '^{"metric"' "$1" | tail -1; }
for s in "" _bf16; do
  d=$G/prof_$T$s
  last_json $d/bench.log > $P/${T}${s}_bench.json
  last_json $d/prof.log > $P/${T}${s}_bench_profiled.json
  cp $d/trace/run_kernel_stats.csv $P/${T}${s}_kernel_stats.csv
  cp $d/pmc_summary.txt $P/${T}${s}_pmc_summary.txt
  cp $d/${T}${s}_pmc.json $P/${T}${s}_pmc.json
done
cp $G/prof_$T/hbm_traffic.json $G/prof_${T}_bf16/hbm_traffic_bf16.json $P/
last_json $G/ctc_$T/ctc.log > $P/${T}_ctc.json
last_json $G/ctc_$T/ctc_fp32.log > $P/${T}_ctc_fp32.json
cp $G/ctc_$T/trace/run_kernel_stats.csv $P/${T}_ctc_kernel_stats.csv
cp $G/ctcpmc_$T/pmc_summary.txt $P/${T}_ctc_pmc_summary.txt
cp $G/ctcpmc_$T/ctc_hbm_traffic.json $P/
cp $G/$T/gputest.log $P/${T}_gputest.log
cp $G/$T/smoke.log $P/${T}_smoke.log
ls $P | grep "^$T"
