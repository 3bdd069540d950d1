"""Per-kernel comparison of two tools/isa_snapshot.sh directories (dev tool).

    python tools/isa_compare.py <before_dir> <after_dir>

Splits each translation unit's device assembly into functions (from one
"-- Begin function" marker to the next) and reports, per unit, the functions only in
one side and those whose instruction text differs.
"""
import os
import re
import sys


def functions(path):
    """name -> instruction text from its "-- Begin function" line to its
    .Lfunc_end label, with the unit-global label numbering (.LBB<f>_<b>)
    normalised to the function."""
    out, name, buf = {}, None, []
    for ln in open(path).read().split("\n"):
        m = re.search(r"-- Begin function (\S+)", ln)
        if m:
            name, buf = m.group(1), []
            continue
        if name and ln.startswith(".Lfunc_end"):
            out[name] = "\n".join(buf)
            name = None
            continue
        if name and "cuid" not in ln:
            ln = ln.split(";")[0].rstrip()   # trailing comments (loop headers name global block numbers)
            buf.append(re.sub(r"\.L(BB|tmp)\d+_?", r".L\1_", ln))
    return out


def main():
    a, b = sys.argv[1], sys.argv[2]
    same = True
    for f in sorted(os.listdir(a)):
        if not f.endswith(".s") or not os.path.exists(os.path.join(b, f)):
            continue
        fa, fb = functions(os.path.join(a, f)), functions(os.path.join(b, f))
        gone, new = sorted(set(fa) - set(fb)), sorted(set(fb) - set(fa))
        changed = sorted(k for k in set(fa) & set(fb) if fa[k] != fb[k])
        if gone or new or changed:
            same = False
        print(f"{f}: {len(fa)} -> {len(fb)} functions, {len(changed)} changed")
        for k in gone:
            print("  removed", k)
        for k in new:
            print("  added  ", k)
        for k in changed:
            print("  CHANGED", k)
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
