"""Instruction-mix summary of one kernel in a hipcc -S output (dev tool).

    python asm_stats.py file.s <substring-of-kernel-name> [--top N]
"""
import re
import sys
from collections import Counter


def kernel_body(text: str, key: str):
    starts = [m for m in re.finditer(r"^(_Z\S+):", text, re.M) if key in m.group(1)]
    if not starts:
        raise SystemExit(f"no kernel matching {key!r}")
    m = starts[0]
    end = text.find(".Lfunc_end", m.end())
    return m.group(1), text[m.end():end]


def main():
    path, key = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    name, body = kernel_body(open(path).read(), key)
    ins = []
    for ln in body.split("\n"):
        ln = ln.strip()
        if not ln or ln.startswith((".", ";", "//")) or ln.endswith(":"):
            continue
        ins.append(ln.split()[0])
    c = Counter(ins)
    cls = Counter()
    for k, v in c.items():
        if k.startswith("v_mfma"):
            cls["mfma"] += v
        elif k.startswith("v_"):
            cls["valu"] += v
        elif k.startswith("s_"):
            cls["salu/ctrl"] += v
        elif k.startswith("ds_"):
            cls["lds"] += v
        elif k.startswith(("global_", "buffer_", "flat_", "scratch_")):
            cls["vmem"] += v
    print(name, "total", len(ins), dict(cls))
    for k, v in c.most_common(top):
        print(f"  {k:32s}{v}")


if __name__ == "__main__":
    main()
