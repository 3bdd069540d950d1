"""Static scan of a gfx950 assembly listing (hipcc --cuda-device-only -S) for
the distance, in wait states, between each MFMA and the first later
instruction that touches its destination registers (the K = 32
question).  Diagnostic tool; nothing in the product or the tests uses it.

    python tools/debug/xdl_hazard_scan.py k32.s [--mnemonic v_mfma_f32_16x16x32_bf16] [--kernel SUBSTR]

The scan follows program order inside one basic block (it stops at a branch or
a label) and counts 1 wait state per instruction, N + 1 for `s_nop N`.  A later
MFMA that takes the destination whole as its C operand (an accumulation chain)
is not a hazard and is skipped.  For every other access it records the kind:
  valu_read / valu_write (WAW) / ds_read_src (address or data of an LDS op) /
  ds_dst (an LDS load overwriting it) / vmem_src / mfma_ab (A/B operand) /
  mfma_c_other (C operand of an MFMA with another destination).
and prints, per kind, the minimum distance seen and how many sites are below a
threshold (default 12: the gfx950 requirement for an 8-pass XDL result read
by a VMEM/LDS/FLAT instruction, cdna_hip_programming.md 5.7 item 2).
"""
from __future__ import annotations

import argparse
import collections
import re
import sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def regs(tok: str):
    out = set()
    for m in REG.finditer(tok):
        f = m.group(1)
        if m.group(4) is not None:
            out.add((f, int(m.group(4))))
        else:
            for r in range(int(m.group(2)), int(m.group(3)) + 1):
                out.add((f, r))
    return out


def split_ops(rest: str):
    rest = rest.split(";")[0]
    parts, depth, cur = [], 0, ""
    for ch in rest:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur.strip())
    return parts


def parse(path, kernel_filter=None):
    funcs = collections.OrderedDict()
    cur = None
    for line in open(path):
        s = line.rstrip("\n")
        if not s.strip() or s.lstrip().startswith((";", "//")):
            continue
        if re.match(r"^[A-Za-z_.$][\w.$]*:", s):
            lab = s.split(":")[0]
            if not lab.startswith("."):
                cur = lab
                funcs.setdefault(cur, [])
            if cur is not None:
                funcs[cur].append(("LABEL", lab, []))
            continue
        if cur is None or not s.startswith((" ", "\t")):
            continue
        t = s.strip()
        if t.startswith("."):
            continue
        mn, _, rest = t.partition(" ")
        funcs[cur].append((mn, rest, split_ops(rest)))
    if kernel_filter:
        funcs = collections.OrderedDict((k, v) for k, v in funcs.items() if kernel_filter in k)
    return funcs


def wait_states(mn, ops):
    if mn == "s_nop":
        try:
            return int(ops[0], 0) + 1
        except (ValueError, IndexError):
            return 1
    return 1


def classify(mn, ops, dst):
    """Kinds of access instruction (mn, ops) makes to the register set dst."""
    kinds = []
    if mn.startswith("v_mfma"):
        d, a, b, c = (regs(o) for o in (ops + ["", "", "", ""])[:4])
        if a & dst or b & dst:
            kinds.append("mfma_ab")
        if c & dst and not (c == dst and d == dst):
            kinds.append("mfma_c_other")   # C operand of an MFMA writing elsewhere (or a partial overlap)
        if d & dst and not (c == dst and d == dst):
            if not (c == d):
                kinds.append("mfma_waw")
        return kinds
    if mn.startswith("ds_"):
        if mn.startswith(("ds_read", "ds_load")) or "_rtn" in mn:
            if ops and regs(ops[0]) & dst:
                kinds.append("ds_dst")
            if any(regs(o) & dst for o in ops[1:]):
                kinds.append("ds_read_src")
        else:
            if any(regs(o) & dst for o in ops):
                kinds.append("ds_read_src")
        return kinds
    if mn.startswith(("buffer_", "global_", "flat_", "scratch_")):
        if "load" in mn:
            if ops and regs(ops[0]) & dst:
                kinds.append("vmem_dst")
            if any(regs(o) & dst for o in ops[1:]):
                kinds.append("vmem_src")
        elif any(regs(o) & dst for o in ops):
            kinds.append("vmem_src")
        return kinds
    if mn.startswith("v_"):
        if mn.startswith(("v_cmp", "v_readfirstlane", "v_readlane")):
            if any(regs(o) & dst for o in ops):
                kinds.append("valu_read")
            return kinds
        if ops and regs(ops[0]) & dst:
            kinds.append("valu_write")
        if any(regs(o) & dst for o in ops[1:]):
            kinds.append("valu_read")
    return kinds


def scan(funcs, mnemonic, horizon=40, thresh=12):
    stats = collections.defaultdict(lambda: [10 ** 9, 0, 0])   # kind -> [min distance, sites, sites < thresh]
    examples = collections.defaultdict(list)
    n_mfma = 0
    for fname, ins in funcs.items():
        for i, (mn, rest, ops) in enumerate(ins):
            if mn != mnemonic:
                continue
            n_mfma += 1
            dst = regs(ops[0])
            dist = 0
            for j in range(i + 1, len(ins)):
                mn2, rest2, ops2 = ins[j]
                if mn2 == "LABEL" or mn2.startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")):
                    break
                dist += 1   # this instruction issues `dist` states after the MFMA
                ks = classify(mn2, ops2, dst)
                for k in ks:
                    st = stats[k]
                    st[0] = min(st[0], dist)
                    st[1] += 1
                    if dist < thresh:
                        st[2] += 1
                        if len(examples[k]) < 4:
                            examples[k].append((fname[:40], dist, f"{mnemonic} {ops[0]}", f"{mn2} {rest2.strip()}"))
                if ks and any(k in ("valu_write", "mfma_waw", "ds_dst", "vmem_dst") for k in ks):
                    break   # the range is overwritten: later reads see the new value
                dist += wait_states(mn2, ops2) - 1
                if dist >= horizon:
                    break
    return n_mfma, stats, examples


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--mnemonic", default="v_mfma_f32_16x16x32_bf16")
    ap.add_argument("--kernel", default=None)
    ap.add_argument("--thresh", type=int, default=12)
    a = ap.parse_args()
    funcs = parse(a.asm, a.kernel)
    n, stats, ex = scan(funcs, a.mnemonic, thresh=a.thresh)
    print(f"{a.asm}: {n} x {a.mnemonic} in {len(funcs)} functions")
    for k, (mn, sites, below) in sorted(stats.items()):
        print(f"  {k:16s} min distance {mn:3d} states, {sites} sites, {below} below {a.thresh}")
        for e in ex[k]:
            print("      ", e)
    return 0


if __name__ == "__main__":
    sys.exit(main())
