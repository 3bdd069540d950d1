"""Instruction mix per code segment between ;WKMARK phase markers (dev tool).

    python tools/asm_phases.py [kernel-substring] [extra hipcc flags...]

Compiles csrc/wk_fused.hip with -DWK_ASM_MARKS (WK_STAMP / WK_FE_HIT become
asm comments), takes the named kernel (default: the fp32 product kernel) and
prints, for each stretch of code between two markers in program order, the
count of VALU / packed-VALU / DPP / MFMA / LDS / VMEM / SALU instructions.
"""
import os
import re
import subprocess
import sys
from collections import Counter

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
key = sys.argv[1] if len(sys.argv) > 1 else "wk_fused_kernelIfLi0ELb0E"
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fno-signed-zeros", "-ffp-contract=fast",
       "-fno-slp-vectorize", "-DWK_ASM_MARKS", "-I", f"{R}/include", "-I", f"{R}/esp32-wake-word_amd/csrc",
       *sys.argv[2:], "--cuda-device-only", "-S", f"{R}/esp32-wake-word_amd/csrc/wk_fused.hip", "-o", "/tmp/asm_phases.s"]


def cls(op, line):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith("v_") and ("_dpp" in op or " row_" in line or "quad_perm" in line):
        return "dpp"
    if op.startswith(("v_log", "v_exp", "v_rcp", "v_sqrt", "v_rsq", "v_sin", "v_cos")):
        return "trans"
    if op.startswith("v_cndmask"):
        return "cndmask"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    subprocess.run(cmd, check=True, capture_output=True)
    text = open("/tmp/asm_phases.s").read()
    m = [x for x in re.finditer(r"^(_Z\S+):", text, re.M) if key in x.group(1)][0]
    body = text[m.end():text.find(".Lfunc_end", m.end())]
    segs, cur, label = [], Counter(), "start"
    for ln in body.split("\n"):
        s = ln.strip()
        mk = re.search(r";WKMARK (\w+)", s)
        if mk:
            segs.append((label + "->" + mk.group(1), cur))
            cur, label = Counter(), mk.group(1)
            continue
        if not s or s.startswith((".", ";", "//")) or s.endswith(":"):
            continue
        cur[cls(s.split()[0], s)] += 1
    segs.append((label + "->end", cur))
    cols = ["valu", "valu_pk", "dpp", "cndmask", "trans", "mfma", "lds", "vmem", "salu", "waitcnt", "nop"]
    print(f"{'segment':18s}" + "".join(f"{c:>8s}" for c in cols) + f"{'total':>8s}")
    for name, c in segs:
        if sum(c.values()) == 0:
            continue
        print(f"{name:18s}" + "".join(f"{c[k]:8d}" for k in cols) + f"{sum(c.values()):8d}")


if __name__ == "__main__":
    main()
