"""Resolve compile-time A/B knobs in a source file (a small unifdef).

    python tools/unifdef_lite.py FILE -DNAME=VALUE ... -UNAME ...

Handles `#if NAME`, `#if !NAME`, `#ifdef NAME`, `#ifndef NAME`, `#elif NAME`,
`#else`, `#endif` and the knob's own default block
(`#ifndef NAME / #define NAME v / #endif`).  Conditions on other macros are
kept as they are.  Used to prune measured-negative variants from the product
sources (git history keeps them).
"""
import re
import sys


def cond_value(expr, defs, undefs):
    expr = expr.split("//")[0].strip()
    m = re.fullmatch(r"(!?)\s*(\w+)", expr)
    if m:
        neg, name = m.groups()
        if name in defs:
            v = defs[name] != "0"
        elif name in undefs:
            v = False
        else:
            return None
        return (not v) if neg else v
    m = re.fullmatch(r"(\w+)\s*==\s*(\d+)", expr)
    if m:
        name, val = m.groups()
        if name in defs:
            return defs[name] == val
        return None
    m = re.fullmatch(r"(\w+)\s*\|\|\s*(\w+)", expr)
    if m:
        a, b = (cond_value(x, defs, undefs) for x in m.groups())
        if a is True or b is True:
            return True
        if a is False and b is False:
            return False
        if a is False:
            return None if b is None else b
        return None
    return None


def process(lines, defs, undefs):
    out = []
    # stack entries: (kind, state) -- kind "keep" (unresolved, lines kept) or
    # "res"; state for res: [taken_any, currently_emitting]
    stack = []

    def emitting():
        return all(e[1][1] for e in stack if e[0] == "res")

    i = 0
    while i < len(lines):
        ln = lines[i]
        s = ln.strip()
        m = re.match(r"#\s*(ifndef|ifdef|if|elif|else|endif)\b\s*(.*)", s)
        if not m:
            if emitting():
                out.append(ln)
            i += 1
            continue
        d, rest = m.groups()
        if d == "ifndef":
            name = rest.split()[0]
            # the knob's own default block
            if (name in defs or name in undefs) and i + 2 < len(lines) and \
                    re.match(r"#\s*define\s+" + name + r"\b", lines[i + 1].strip()) and \
                    lines[i + 2].strip().startswith("#endif"):
                i += 3
                continue
            v = None if name not in defs and name not in undefs else (name in undefs)
        elif d == "ifdef":
            name = rest.split()[0]
            v = None if name not in defs and name not in undefs else (name in defs)
        elif d == "if":
            v = cond_value(rest, defs, undefs)
        if d in ("ifndef", "ifdef", "if"):
            if v is None:
                stack.append(("keep", None))
                if emitting():
                    out.append(ln)
            else:
                stack.append(("res", [v, v]))
        elif d == "elif":
            kind, st = stack[-1]
            if kind == "keep":
                if emitting():
                    out.append(ln)
            else:
                v = cond_value(rest, defs, undefs)
                if v is None:
                    raise SystemExit(f"line {i+1}: unresolved #elif after a resolved #if")
                st[1] = (not st[0]) and v
                st[0] = st[0] or v
        elif d == "else":
            kind, st = stack[-1]
            if kind == "keep":
                if emitting():
                    out.append(ln)
            else:
                st[1] = not st[0]
                st[0] = True
        elif d == "endif":
            kind, st = stack.pop()
            if kind == "keep" and emitting():
                out.append(ln)
        i += 1
    assert not stack, "unbalanced conditionals"
    return out


def main():
    path = sys.argv[1]
    defs, undefs = {}, set()
    for a in sys.argv[2:]:
        if a.startswith("-D"):
            k, _, v = a[2:].partition("=")
            defs[k] = v or "1"
        elif a.startswith("-U"):
            undefs.add(a[2:])
    lines = open(path).read().split("\n")
    out = process(lines, defs, undefs)
    open(path, "w").write("\n".join(out))


if __name__ == "__main__":
    main()
