#!/usr/bin/env python3
"""Minimal unifdef: resolve the preprocessor conditionals that depend only on
the given macros, keep every other conditional as it is.

    tools/unifdef.py -DFC_STUB=0 -UFC_STAMPS < in.hip > out.hip

Used to keep the attribution builds (phase stubs, clock stamps) out of the
product source: the product holds the resolved text, and tools/attribution/
keeps each variant as a patch against it (tools/attribution/apply.sh).
"""
import re
import sys

DIRECTIVE = re.compile(r"^\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)$")
IDENT = re.compile(r"[A-Za-z_]\w*")


def parse_args(argv):
    known = {}
    for a in argv:
        if a.startswith("-D"):
            k, _, v = a[2:].partition("=")
            known[k] = v if v else "1"
        elif a.startswith("-U"):
            known[a[2:]] = None
    return known


def evaluate(kind, expr, known):
    """True / False when decided by the known macros alone, None otherwise."""
    expr = expr.split("//")[0].strip()
    if kind in ("ifdef", "ifndef"):
        name = expr.split()[0]
        if name not in known:
            return None
        defined = known[name] is not None
        return defined if kind == "ifdef" else not defined
    names = set(IDENT.findall(expr)) - {"defined"}
    unknown = sorted(names - set(known))
    if not names or len(unknown) > 4 or unknown == sorted(names):
        return None
    if unknown:
        # decided when every value of the unknown macros (0 / 1 each) agrees
        outs = set()
        for bits in range(1 << len(unknown)):
            trial = dict(known)
            trial.update({u: str((bits >> i) & 1) for i, u in enumerate(unknown)})
            outs.add(evaluate(kind, expr, trial))
        return outs.pop() if len(outs) == 1 else None
    py = re.sub(r"defined\s*\(?\s*(\w+)\s*\)?",
                lambda m: "1" if known.get(m.group(1)) is not None else "0", expr)
    py = IDENT.sub(lambda m: m.group(0) if m.group(0) in ("and", "or", "not")
                   else str(known.get(m.group(0)) or 0), py)
    py = py.replace("&&", " and ").replace("||", " or ").replace("!", " not ").replace(" not =", "!=")
    return bool(eval(py, {}, {}))


def unifdef(lines, known):
    out = []
    # stack entries: [mode, taken]; mode "keep" = directive kept (unknown),
    # "resolved" = this conditional is being removed; taken = a branch was
    # already selected; active = emitting lines of the current branch
    stack = []

    def active():
        return all(e["active"] for e in stack)

    for line in lines:
        m = DIRECTIVE.match(line)
        if not m:
            if active():
                out.append(line)
            continue
        kind, rest = m.group(1), m.group(2)
        if kind in ("if", "ifdef", "ifndef"):
            v = evaluate(kind, rest, known) if active() else None
            if v is None:
                stack.append({"resolved": False, "taken": False, "active": True, "emit": active()})
                if active():
                    out.append(line)
            else:
                stack.append({"resolved": True, "taken": v, "active": v, "emit": True})
            continue
        top = stack[-1]
        if kind == "elif":
            if top["resolved"]:
                if top["taken"]:
                    top["active"] = False
                    continue
                v = evaluate("if", rest, known)
                if v is None:
                    # the first undecided branch becomes a plain #if
                    top.update(resolved=False, active=True, taken=False)
                    out.append(line.replace("#elif", "#if", 1))
                else:
                    top["active"] = v
                    top["taken"] = v
            else:
                v = evaluate("if", rest, known)
                if v is False:
                    top["active"] = False
                    top["skip_elif"] = True
                    continue
                top["active"] = True
                if top["emit"]:
                    out.append(line)
            continue
        if kind == "else":
            if top["resolved"]:
                top["active"] = not top["taken"]
                top["taken"] = True
            else:
                top["active"] = True
                if top["emit"]:
                    out.append(line)
            continue
        if kind == "endif":
            e = stack.pop()
            if not e["resolved"] and e["emit"]:
                out.append(line)
    assert not stack, "unbalanced conditionals"
    return out


def main():
    known = parse_args(sys.argv[1:])
    sys.stdout.write("".join(unifdef(sys.stdin.readlines(), known)))


if __name__ == "__main__":
    main()
