"""Resolves preprocessor conditionals on a given set of macros (a small
unifdef): used once to strip rejected variants and timing ablations out of
the product kernels, and to regenerate tools/patches/*.patch, which put the
ablation hooks back into a scratch copy for tools/build_variants.sh.

    python tools/unifdef.py -DNAME[=V] ... -FNAME=V ... -UNAME ... < in > out

-D: the macro is defined (its own `#define` defaults are dropped); -F: a fixed
value whose default `#ifndef NAME / #define NAME v / #endif` stays as a plain
`#define` (the guard goes, the value is the product's); -U: undefined.

Only conditionals whose expression is decided by the given macros are
resolved (#if / #ifdef / #ifndef / #elif / #else / #endif, with !, &&, ||,
defined(), integer values and parentheses); every other conditional and line
is kept as is. `#define X` / `#ifndef X #define X v #endif` defaults of a
resolved macro are dropped when the macro is given.
"""
import re
import sys

TOKEN = re.compile(r"\s*(defined|\(|\)|!|&&|\|\||[A-Za-z_]\w*|\d+)")


class Unknown(Exception):
    pass


def evaluate(expr, defs, undefs):
    toks = TOKEN.findall(expr.split("//")[0].split("/*")[0])
    pos = [0]

    def peek():
        return toks[pos[0]] if pos[0] < len(toks) else None

    def take():
        pos[0] += 1
        return toks[pos[0] - 1]

    def atom():
        t = take()
        if t == "!":
            v = atom()
            return None if v is None else int(not v)
        if t == "(":
            v = orx()
            take()
            return v
        if t == "defined":
            paren = peek() == "("
            if paren:
                take()
            name = take()
            if paren:
                take()
            if name in defs:
                return 1
            if name in undefs:
                return 0
            return None
        if t.isdigit():
            return int(t)
        if t in defs:
            return int(defs[t])
        if t in undefs:
            return 0
        return None

    def andx():
        v = atom()
        while peek() == "&&":
            take()
            w = atom()
            v = 0 if (v == 0 or w == 0) else (None if v is None or w is None else int(v and w))
        return v

    def orx():
        v = andx()
        while peek() == "||":
            take()
            w = andx()
            v = 1 if (v or w) else (None if v is None or w is None else 0)
        return v
    return orx()


def process(lines, defs, undefs, fixed=()):
    out = []
    # stack entries: [mode, taken] ; mode: "keep" (directive kept) / "res" (resolved)
    # emit: whether lines of the current branch are emitted
    stack = []
    emit = True
    known = set(defs) | set(undefs)
    i = 0
    while i < len(lines):
        line = lines[i]
        m = re.match(r"\s*#\s*(ifdef|ifndef|if|elif|else|endif)\b(.*)", line)
        d = re.match(r"\s*#\s*define\s+(\w+)", line)
        if d and d.group(1) in known and d.group(1) not in fixed and emit:
            # a default of a resolved macro: dropped
            i += 1
            continue
        if not m:
            if emit:
                out.append(line)
            i += 1
            continue
        kw, rest = m.group(1), m.group(2).strip()
        if kw in ("ifdef", "ifndef", "if"):
            if kw == "ifdef":
                name = rest.split()[0]
                v = 1 if name in defs else 0 if name in undefs else None
            elif kw == "ifndef":
                name = rest.split()[0]
                v = 1 if name in fixed else 0 if name in defs else 1 if name in undefs else None
            else:
                v = evaluate(rest, defs, undefs)
            parent = emit
            if v is None:
                stack.append({"mode": "keep", "parent": parent, "taken": None})
                if emit:
                    out.append(line)
            else:
                stack.append({"mode": "res", "parent": parent, "taken": bool(v)})
                emit = parent and bool(v)
        elif kw == "elif":
            top = stack[-1]
            if top["mode"] == "keep":
                if top["parent"]:
                    out.append(line)
            else:
                v = evaluate(rest, defs, undefs)
                if v is None:
                    raise Unknown(f"line {i + 1}: #elif on an unresolved macro after a resolved #if")
                emit = top["parent"] and not top["taken"] and bool(v)
                top["taken"] = top["taken"] or bool(v)
        elif kw == "else":
            top = stack[-1]
            if top["mode"] == "keep":
                if top["parent"]:
                    out.append(line)
            else:
                emit = top["parent"] and not top["taken"]
                top["taken"] = True
        else:  # endif
            top = stack.pop()
            if top["mode"] == "keep" and top["parent"]:
                out.append(line)
            emit = top["parent"]
        i += 1
    assert not stack, "unbalanced conditionals"
    return out


def main(argv):
    defs, undefs, fixed = {}, set(), set()
    for a in argv:
        if a.startswith("-D") or a.startswith("-F"):
            k, _, v = a[2:].partition("=")
            defs[k] = v or "1"
            if a.startswith("-F"):
                fixed.add(k)
        elif a.startswith("-U"):
            undefs.add(a[2:])
    sys.stdout.write("".join(process(sys.stdin.readlines(), defs, undefs, fixed)))


if __name__ == "__main__":
    main(sys.argv[1:])
