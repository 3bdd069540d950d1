#!/bin/bash
# Instruction census of the fused kernel by class (run on the GPU box via gpurun):
#   bash tools/pmc_census.sh <outdir> [bench args...]
# Two rocprofv3 --pmc passes over a short bench.py run (8 SQ counters each);
# summarise with:  python tools/pmc_census.py <outdir>
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(realpath -m "${1:-$R/gpurun_out/census}"); shift
ARGS=${@:-"--steps 2 --warmup 1 --no-cpu-baseline"}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/c$i" -o run --output-format csv -- python3 "$R/bench.py" $ARGS \
    > "$OUT/c$i.log" 2>&1 || { echo "census pass $i ($grp) failed rc=$?"; tail -5 "$OUT/c$i.log"; exit 1; }
  echo "census pass $i ok: $grp"
done <<'GROUPS'
SQ_INSTS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_MFMA
SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MFMA_F32 SQ_WAVES
SQ_INSTS_VALU_FLOPS_FP32 SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
GROUPS
