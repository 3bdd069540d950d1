#!/bin/bash
# Round-6 evidence in one GPU call (through gpurun): the -m gpu suite and smoke(),
# then the fp32 and bf16 profile bundles (tools/profile_round.sh: bench line with
# configs 4/5/3, rocprofv3 kernel stats, PMC, HBM traffic) and the config-5
# bundle with its PMC.  Each GPU step has its own time limit; the first failure ends the call.
#   bash tools/round6_bundle.sh <tag>
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
T=${1:?tag}
O=$R/gpurun_out/$T
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gputest.log" 2>&1
rc=$?; tail -3 "$O/gputest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
cat "$O/smoke.log"
bash tools/profile_round.sh "$T" || exit $?
bash tools/profile_round.sh "${T}_bf16" --precision bf16 || exit $?
bash tools/ctc_bundle.sh "$T" || exit $?
timeout -k 10 900 bash tools/ctc_pmc.sh "$T" > "$O/ctc_pmc.log" 2>&1 || exit $?
echo done
