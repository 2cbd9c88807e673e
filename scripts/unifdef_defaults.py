"""Resolve the measured-variant switches of csrc/*.hip to their defaults (a small unifdef).

Every `#ifndef DAUC_X / #define DAUC_X v / #endif` default block of a known switch is dropped,
`#if / #ifdef / #ifndef / #elif / #else / #endif` groups whose conditions use only known
switches are resolved, and the remaining uses of a switch are replaced by its value. Conditions
that mention anything else (DAUC_TUNING, include guards) are left untouched.

    python scripts/unifdef_defaults.py distributedauc_amd/csrc/*.hip
"""
from __future__ import annotations

import re
import sys

DEFAULTS = {
    "DAUC_COMPACT_WIDE_THREADS": 256, "DAUC_COMPACT_BATCH": 8, "DAUC_SORT_PER_THREAD": 8,
    "DAUC_QUERY_MAX_SPLIT": 40000, "DAUC_QUERY_BLOCKS_PER_CU": 1, "DAUC_ABLATE": 0, "DAUC_QUERY_LOCKSTEP": 0,
    "DAUC_TREE_ARITY": 5, "DAUC_TREE_TOP_LEVELS": 0, "DAUC_TREE_STEP": 0, "DAUC_QUERY_PIPE": 0,
    "DAUC_QUERY_PIPE_U": 2, "DAUC_CI_WIN_NT": 0, "DAUC_CI_ABLATE": 0, "DAUC_CI_PIPE": 1,
    "DAUC_CI_PHASED": 1, "DAUC_CI_U": 1, "DAUC_CI_ABLATE2": 0, "DAUC_CI_LATEWIN": 0, "DAUC_CI_MED3": 0,
    "DAUC_CI_W2": 1, "DAUC_CI_COUNT3": 0, "DAUC_CI_DEPTH": 1, "DAUC_SURROGATE_SLOTS": 8,
    "DAUC_SURROGATE_BPC": 2, "DAUC_SURROGATE_NTSTORE": 1, "DAUC_TAIL_WAVES": 1, "DAUC_TAIL_PREPOLL": 0,
    "DAUC_SURROGATE_TAIL_REDUCERS": 64, "DAUC_TAIL_LAG": 4096, "DAUC_BK_X": 0,
}
IDENT = re.compile(r"\b[A-Za-z_]\w*\b")


def evaluate(expr: str):
    """The value of a #if expression over known switches, or None if it mentions anything else."""
    expr = re.sub(r"//.*", "", expr).strip()
    e = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "1" if m.group(1) in DEFAULTS else f"@{m.group(1)}", expr)
    e = re.sub(r"defined\s+(\w+)", lambda m: "1" if m.group(1) in DEFAULTS else f"@{m.group(1)}", e)
    if "@" in e:
        return None
    names = set(IDENT.findall(e))
    if not names <= set(DEFAULTS):
        return None
    for n in sorted(names, key=len, reverse=True):
        e = re.sub(rf"\b{n}\b", str(DEFAULTS[n]), e)
    e = e.replace("&&", " and ").replace("||", " or ").replace("!", " not ").replace(" not =", "!=")
    return bool(eval(e, {}, {}))  # noqa: S307 (integer literals and operators only)


def process(text: str) -> str:
    lines = text.split("\n")
    # drop the default blocks: #ifndef X / #define X v [comment] / #endif
    out = []
    i = 0
    while i < len(lines):
        m = re.match(r"\s*#ifndef\s+(DAUC_\w+)\s*$", lines[i])
        if m and m.group(1) in DEFAULTS and i + 2 < len(lines) and re.match(
                rf"\s*#define\s+{m.group(1)}\b", lines[i + 1]):
            j = i + 2
            while not re.match(r"\s*#endif", lines[j]):  # a continued comment line
                j += 1
            i = j + 1
            continue
        out.append(lines[i])
        i += 1
    lines = out
    # resolve conditional groups (a stack of [known, taking, any_taken])
    out, stack = [], []

    def active():
        return all(f[1] for f in stack if f[0])

    for ln in lines:
        d = re.match(r"\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)", ln)
        if not d:
            if active():
                out.append(ln)
            continue
        kind, rest = d.group(1), d.group(2)
        if kind in ("if", "ifdef", "ifndef"):
            if kind == "if":
                v = evaluate(rest)
            else:
                name = rest.strip().split()[0]
                v = (name in DEFAULTS) if name in DEFAULTS else None
                if v is not None and kind == "ifndef":
                    v = not v
            if v is None:
                stack.append([False, True, True])
                if active():
                    out.append(ln)
            else:
                stack.append([True, v, v])
        elif kind == "elif":
            f = stack[-1]
            if not f[0]:
                if active():
                    out.append(ln)
                continue
            v = evaluate(rest)
            if v is None:
                raise ValueError(f"unresolvable #elif after a resolved #if: {ln}")
            f[1] = (not f[2]) and v
            f[2] = f[2] or v
        elif kind == "else":
            f = stack[-1]
            if not f[0]:
                if active():
                    out.append(ln)
                continue
            f[1] = not f[2]
            f[2] = True
        else:
            f = stack.pop()
            if not f[0] and active():
                out.append(ln)
    text = "\n".join(out)
    for n in sorted(DEFAULTS, key=len, reverse=True):
        text = re.sub(rf"\b{n}\b", str(DEFAULTS[n]), text)
    return text


if __name__ == "__main__":
    for path in sys.argv[1:]:
        src = open(path).read()
        new = process(src)
        if new != src:
            open(path, "w").write(new)
            print(f"{path}: {src.count(chr(10))} -> {new.count(chr(10))} lines")
