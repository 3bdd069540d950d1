#!/bin/bash
# LDS bank conflicts of the fused GRU per access site: one rocprofv3 --pmc pass
# over bench_ctc.py per variants/var_gl<mask> build (WK_GRU_LDSABL bitmask:
# 1 x-tile writes, 2 x-tile reads, 4 state reads, 8 state writes, 16 output
# copy reads, 32 layer-1 W reads; timing/counter diagnostics, wrong results).
#   bash tools/debug/gru_lds_abl.sh <mask...>   (through gpurun)
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/gru_lds
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for m in "$@"; do
  WAKEWORD_LIB=$R/variants/var_gl$m/libwakeword.so timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS \
    -d "$O/m$m" -o run --output-format csv -- python3 "$R/bench_ctc.py" --steps 1 --warmup 1 --no-cpu-baseline > "$O/m$m.log" 2>&1 || { echo "mask $m failed"; tail -3 "$O/m$m.log"; exit 1; }
  python3 - "$O/m$m" "$m" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv") + glob.glob(sys.argv[1] + "/run_counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        if "gru16x" in row["Kernel_Name"]:
            k = "L0" if "ILi128" in row["Kernel_Name"] else "L1"
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(acc):
    c = {n: sum(v) / len(v) for n, v in acc[k].items()}
    print(f"mask {sys.argv[2]:>3} {k}: conflict {c.get('SQ_LDS_BANK_CONFLICT', 0):.3e} active {c.get('SQ_LDS_IDX_ACTIVE', 0):.3e} "
          f"insts {c.get('SQ_INSTS_LDS', 0):.3e} share {c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c.get('SQ_LDS_IDX_ACTIVE', 1), 1):.3f}")
PY
done
