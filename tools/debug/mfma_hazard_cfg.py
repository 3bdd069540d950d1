"""Like mfma_hazard_scan.py, but follows the control flow (fall-through and
branch targets, loops included) from every MFMA for up to LIMIT wait states,
reporting the minimum distance to any instruction that reads or overwrites
the MFMA's destination VGPRs (a same-accumulator MFMA chain excluded).
Diagnostic for the K=32 bf16 MFMA corruption."""
import sys
from collections import Counter, defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from mfma_hazard_scan import regs  # noqa: E402

LIMIT = 24


def load(path, kern):
    lines = open(path).read().splitlines()
    st = next(i for i, l in enumerate(lines) if l.startswith(kern))
    en = next(i for i in range(st + 1, len(lines)) if "-- End function" in lines[i] or lines[i].startswith("\t.size"))
    ins, labels = [], {}
    for ln in lines[st + 1:en]:
        s = ln.split(";")[0].strip()
        if s.endswith(":"):
            labels[s[:-1]] = len(ins)
            continue
        if not s or s.startswith("."):
            continue
        parts = s.split(None, 1)
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        ins.append((parts[0], s, ops))
    return ins, labels


def succ(ins, labels, k):
    op, _, ops = ins[k]
    if op == "s_branch":
        return [labels[ops[0]]]
    if op.startswith("s_cbranch"):
        return [k + 1, labels[ops[0]]]
    if op in ("s_endpgm", "s_setpc_b64"):
        return []
    return [k + 1]


def cost(ins, k):
    op, _, ops = ins[k]
    return int(ops[0], 0) + 1 if op == "s_nop" else 1


def main():
    path, kern = sys.argv[1], sys.argv[2]
    only = sys.argv[3] if len(sys.argv) > 3 else "bf16"
    ins, labels = load(path, kern)
    hist = defaultdict(Counter)
    ex = defaultdict(list)
    for k, (op, text, ops) in enumerate(ins):
        if not op.startswith("v_mfma") or only not in op:
            continue
        dst = regs(ops[0])
        best = {}
        stack = [(j, 0) for j in succ(ins, labels, k)]
        while stack:
            j, d = stack.pop()
            if j >= len(ins) or d > LIMIT or best.get(j, 1 << 30) <= d:
                continue
            best[j] = d
            op2, text2, ops2 = ins[j]
            stop = False
            if ops2 and op2 != "s_nop":
                w = regs(ops2[0])
                r = set().union(*[regs(o) for o in ops2[1:]]) if len(ops2) > 1 else set()
                if op2.startswith(("ds_write", "buffer_store", "global_store", "ds_store")):
                    r, w = r | w, set()
                if dst & (r | w):
                    stop = True
                    if op2.startswith("v_mfma") and regs(ops2[3]) == dst and not (dst & (regs(ops2[1]) | regs(ops2[2]))):
                        kind = "mfma-srcC-full"
                    elif op2.startswith("v_mfma"):
                        kind = "mfma-other"
                    else:
                        kind = ("read:" if dst & r else "write:") + op2.split("_")[0]
                    hist[kind][d] += 1
                    ex[kind].append((d, text, text2))
            if not stop:
                stack += [(s, d + cost(ins, j)) for s in succ(ins, labels, j)]
    for kind in sorted(hist):
        print(kind, "min", min(hist[kind]), sorted(hist[kind].items())[:10])
        for d, a, b in sorted(ex[kind])[:3]:
            print("    ", d, "|", a, "->", b)


if __name__ == "__main__":
    main()
