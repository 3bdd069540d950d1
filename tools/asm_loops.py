"""Instruction mix of each loop (back-edge region) of one kernel in a -S file (dev tool).

    python tools/asm_loops.py file.s <kernel-substring> [min_instructions]
"""
import re
import sys
from collections import Counter



def cls(op, line):
    """Instruction class of one ISA line (op = its mnemonic)."""
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


path, key = sys.argv[1], sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 200
text = open(path).read()
m = [x for x in re.finditer(r"^(_Z\S+):", text, re.M) if key in x.group(1)][0]
body = text[m.end():text.find(".Lfunc_end", m.end())].split("\n")
labels, ins = {}, []
for ln in body:
    s = ln.strip()
    lm = re.match(r"^(\.LBB\w+):", s)
    if lm:
        labels[lm.group(1)] = len(ins)
        continue
    if not s or s.startswith((".", ";", "//")) or s.endswith(":"):
        continue
    ins.append(s)
for i, s in enumerate(ins):
    mm = re.match(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", s)
    if not mm:
        continue
    tgt = mm.group(1) or mm.group(2)
    j = labels.get(tgt)
    if j is None or j > i or i - j < mn:
        continue
    c = Counter(cls(x.split()[0], x) for x in ins[j:i + 1])
    print(f"loop {tgt} [{j}..{i}] {i - j + 1} instr: " + " ".join(f"{k}={v}" for k, v in c.most_common()))
