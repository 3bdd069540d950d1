#!/bin/bash
# rocprofv3 PMC passes for the bench workload (run on the GPU box via gpurun).
# Each counter group is its own rocprofv3 run (no --pmc with trace domains).
#   bash tools/profile_pmc.sh <outdir> [bench args...]
# (PMC_BENCH=bench_ctc.py profiles the CTC bench instead of bench.py)
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$R/gpurun_out/pmc}; shift
ARGS=${@:-"--steps 2 --warmup 1 --no-cpu-baseline"}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/${PMC_BENCH:-bench.py}" $ARGS \
    > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($grp) failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok: $grp"
done <<'GROUPS'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
GROUPS
