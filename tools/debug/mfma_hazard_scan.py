"""Scan a gfx950 .s file for the distance (in wait states: 1 per instruction,
N+1 per s_nop N) between each MFMA and the first later instruction of the same
basic block that reads or overwrites the MFMA's destination VGPRs (other than
an MFMA taking them as its accumulator).  Diagnostic for the K=32 bf16 MFMA
corruption.

    python tools/debug/mfma_hazard_scan.py file.s [kernel-substring]
"""
import re
import sys
from collections import Counter, defaultdict

REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")


def regs(opnd):
    out = set()
    for m in REG.finditer(opnd):
        if m.group(1):
            out |= {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


def parse(lines):
    ins = []
    for ln in lines:
        s = ln.split(";")[0].strip()
        if not s or s.startswith(".") or s.endswith(":"):
            ins.append(("LABEL", "", []) if s.endswith(":") else None)
            continue
        parts = s.split(None, 1)
        op = parts[0]
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        ins.append((op, s, ops))
    return [i for i in ins if i is not None]


def main():
    path = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else None
    lines = open(path).read().splitlines()
    if kern:
        st = next(i for i, l in enumerate(lines) if l.startswith(kern) or (kern in l and l.endswith(":") and not l.startswith("\t")))
        en = next(i for i in range(st + 1, len(lines)) if lines[i].startswith("\t.size") or "-- End function" in lines[i])
        lines = lines[st:en]
    ins = parse(lines)
    hist = defaultdict(Counter)
    worst = defaultdict(list)
    for k, (op, text, ops) in enumerate(ins):
        if not op.startswith("v_mfma"):
            continue
        dst = regs(ops[0])
        dist = 0
        for op2, text2, ops2 in ins[k + 1:]:
            if op2 == "LABEL" or op2.startswith("s_cbranch") or op2 == "s_branch" or op2 == "s_setpc_b64":
                break
            if op2 == "s_nop":
                dist += int(ops2[0], 0) + 1
                continue
            if not ops2:
                dist += 1
                continue
            w = regs(ops2[0])
            r = set().union(*[regs(o) for o in ops2[1:]]) if len(ops2) > 1 else set()
            if op2.startswith("ds_write") or op2.startswith("buffer_store") or op2.startswith("global_store") or op2.startswith("ds_store"):
                r |= w
                w = set()
            hit_r, hit_w = dst & r, dst & w
            if op2.startswith("v_mfma"):
                if hit_w and regs(ops2[3]) == dst and not (dst & set().union(*[regs(o) for o in ops2[1:3]])):
                    break   # same-accumulator chain (hardware-forwarded)
                if hit_r or hit_w:
                    hist[(op, "mfma-src" if hit_r else "mfma-waw")][dist] += 1
                    break
            elif hit_r or hit_w:
                kind = ("read" if hit_r else "write") + ":" + op2.split("_")[0]
                hist[(op, kind)][dist] += 1
                worst[(op, kind)].append((dist, text, text2))
                break
            dist += 1
    for key in sorted(hist):
        c = hist[key]
        print(key, "min", min(c), "counts", sorted(c.items())[:8])
        for d, a, b in sorted(worst[key])[:2]:
            print("    ", d, "|", a, "->", b)


if __name__ == "__main__":
    main()
