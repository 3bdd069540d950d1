#!/bin/bash
# Ad-hoc rocprofv3 PMC passes (one counter group per run, no trace domains):
#   bash tools/debug/pmc_groups.sh <outdir> <groups-file> [bench args...]
# Environment (e.g. WAKEWORD_FUSED_EXP, honoured by -DWK_DIAG builds only) passes through to bench.py.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$(realpath -m "$1"); GF=$(realpath "$2"); shift 2
ARGS=${@:-"--steps 2 --warmup 1 --no-cpu-baseline"}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/bench.py" $ARGS \
    > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($grp) failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
done < "$GF"
python3 "$R/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt" && echo ok
