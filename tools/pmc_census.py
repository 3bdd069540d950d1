"""Per-window instruction census of the fused kernel from tools/pmc_census.sh output.

    python tools/pmc_census.py <outdir> [--batch 65536] [--json out.json]

Counter means per dispatch of wk_fused_kernel<...> (warm-up dispatches
included: every dispatch is the same batch), divided by the batch: the
instructions the SIMDs issue per window, by class.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    B = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 65536
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if "wk_fused_kernel" not in row["Kernel_Name"]:
                continue
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in vals.items()}
    per = {k: v / B for k, v in m.items()}
    out = {"batch": B, "per_window": per, "per_launch": m}
    if "SQ_INSTS_VALU" in per and "SQ_INSTS_LDS" in per:
        out["valu_plus_lds_per_window"] = per["SQ_INSTS_VALU"] + per["SQ_INSTS_LDS"]
    if "SQ_INSTS_VALU_FLOPS_FP32" in per:
        out["fp32_vector_flop_per_window"] = per["SQ_INSTS_VALU_FLOPS_FP32"]
    if "SQ_WAVE_CYCLES" in m:
        for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if c in m:
                out["share_" + c] = m[c] / m["SQ_WAVE_CYCLES"]
    # SIMD-time shares (counters summed over the chip): SQ_ACTIVE_INST_* and
    # SQ_WAVE_CYCLES count quad-cycles per wave; SQ_VALU_MFMA_BUSY_CYCLES counts
    # cycles; GRBM_GUI_ACTIVE / 8 XCDs = the kernel's cycles; 1,024 SIMDs.
    if "GRBM_GUI_ACTIVE" in m:
        kc = m["GRBM_GUI_ACTIVE"] / 8.0
        simd_cycles = 1024 * kc
        out["kernel_cycles"] = kc
        if "SQ_ACTIVE_INST_VALU" in m:
            out["simd_share_valu_active"] = 4 * m["SQ_ACTIVE_INST_VALU"] / simd_cycles
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            out["simd_share_mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
        if "SQ_ACTIVE_INST_ANY" in m:
            out["simd_share_any_active"] = 4 * m["SQ_ACTIVE_INST_ANY"] / simd_cycles
    for k in sorted(per):
        print(f"{k:28s} {per[k]:12.1f} per window")
    for k, v in out.items():
        if k.startswith(("share_", "valu_plus", "fp32_vector", "simd_share", "kernel_cycles")):
            print(f"{k:28s} {v:12.4f}")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
