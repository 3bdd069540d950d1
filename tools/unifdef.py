"""Resolve preprocessor conditionals on a set of known macros (dev tool).

    python tools/unifdef.py file -DNAME=VALUE ... -UNAME ... [--drop-defaults]

Every #if / #ifdef / #ifndef / #elif / #else / #endif group whose condition
mentions only known macros (plus `defined(...)` of known ones) is evaluated
and replaced by the taken branch; groups mentioning any unknown macro are kept
(their nested known groups are still resolved).  --drop-defaults also removes
`#ifndef NAME / #define NAME v / #endif` default blocks of known macros, and
--subst replaces the remaining uses of known macros in code by their values.
The file is rewritten in place.  Used to fold measured-and-rejected
experiment switches out of the product sources; the product ISA is checked
unchanged with tools/isa_snapshot.sh.
"""
import re
import sys


def parse_args(argv):
    path = argv[1]
    known = {}
    for a in argv[2:]:
        if a.startswith("-D"):
            k, _, v = a[2:].partition("=")
            known[k] = v if v else "1"
        elif a.startswith("-U"):
            known[a[2:]] = None   # undefined
    return path, known, "--drop-defaults" in argv


def cond_value(kind, expr, known):
    """True/False if decidable from known macros, else None."""
    expr = expr.split("//")[0].split("/*")[0].strip()
    if kind in ("ifdef", "ifndef"):
        name = expr.split()[0]
        if name not in known:
            return None
        d = known[name] is not None
        return d if kind == "ifdef" else not d
    names = set(re.findall(r"\b[A-Z_][A-Z0-9_]*\b", expr)) - {"defined"}
    if not names or any(n not in known for n in names):
        return None
    e = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "1" if known[m.group(1)] is not None else "0", expr)
    e = re.sub(r"defined\s+(\w+)", lambda m: "1" if known[m.group(1)] is not None else "0", e)
    for n in names:
        v = known[n]
        e = re.sub(rf"\b{n}\b", "0" if v is None else v, e)
    e = e.replace("&&", " and ").replace("||", " or ").replace("!", " not ").replace(" not =", "!=")
    return bool(eval(e))


def main():
    path, known, drop_defaults = parse_args(sys.argv)
    lines = open(path).read().split("\n")
    out = []
    # stack entries: [mode, taken, emitting_parent]
    #   mode "keep": an undecidable group, lines passed through
    #   mode "fold": a decided group; taken = a branch was already chosen; active = current branch emits
    stack = []

    def emitting():
        return all(s["active"] for s in stack)

    i = 0
    while i < len(lines):
        ln = lines[i]
        m = re.match(r"^\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)$", ln)
        if drop_defaults and m and m.group(1) == "ifndef":
            name = m.group(2).split()[0]
            if name in known and i + 2 < len(lines) and re.match(rf"^\s*#\s*define\s+{name}\b", lines[i + 1]) \
                    and re.match(r"^\s*#\s*endif", lines[i + 2]):
                i += 3
                continue
        if not m:
            if emitting():
                out.append(ln)
            i += 1
            continue
        kind, rest = m.group(1), m.group(2)
        if kind in ("if", "ifdef", "ifndef"):
            v = cond_value(kind, rest, known)
            if v is None:
                stack.append({"mode": "keep", "active": True})
                if emitting():
                    out.append(ln)
            else:
                stack.append({"mode": "fold", "active": v, "taken": v})
        elif kind == "elif":
            top = stack[-1]
            if top["mode"] == "keep":
                v = cond_value("if", rest, known)
                if v is None:
                    if all(s["active"] for s in stack[:-1]):
                        out.append(ln)
                else:
                    # an undecidable group with a decidable elif: keep it textual (rare); emit as-is
                    if all(s["active"] for s in stack[:-1]):
                        out.append(ln)
            else:
                if top["taken"]:
                    top["active"] = False
                else:
                    v = cond_value("if", rest, known)
                    if v is None:
                        raise SystemExit(f"{path}:{i + 1}: undecidable #elif in a folded group")
                    top["active"] = v
                    top["taken"] = v
        elif kind == "else":
            top = stack[-1]
            if top["mode"] == "keep":
                if all(s["active"] for s in stack[:-1]):
                    out.append(ln)
            else:
                top["active"] = not top["taken"]
                top["taken"] = True
        else:  # endif
            top = stack.pop()
            if top["mode"] == "keep" and emitting():
                out.append(ln)
        i += 1
    if "--subst" in sys.argv:   # remaining uses of known macros in code -> their values
        for k, v in known.items():
            if v is None:
                continue
            out = [ln if re.match(r"^\s*#", ln) else re.sub(rf"\b{k}\b", v, ln) for ln in out]
    open(path, "w").write("\n".join(out))


if __name__ == "__main__":
    main()
