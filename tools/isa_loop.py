#!/usr/bin/env python3
"""Instruction mix of the loops of one kernel in a device assembly file: for every loop header
label, the static instruction counts between it and its back-edge branch.

    python tools/isa_loop.py <file.s> <symbol-substring> [max-loops]
"""
import collections
import re
import sys


def main(path, sub, nmax=4):
    s = open(path).read()
    m = next(m for m in re.finditer(r"^(_Z\S+):[^\n]*\n", s, re.M) if sub in m.group(1))
    body = s[m.end():s.index(".Lfunc_end", m.end())].split("\n")
    heads = [(k, l.split(":")[0]) for k, l in enumerate(body) if "Loop Header" in l]
    print(m.group(1), len(heads), "loops")
    for k, lab in heads[:int(nmax)]:
        ends = [q for q, l in enumerate(body) if lab in l and ("s_branch" in l or "s_cbranch" in l) and q > k]
        if not ends:
            continue
        loop = body[k:max(ends)]
        c = collections.Counter(l.split()[0] for l in loop
                                if l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;"))
        tot = sum(c.values())
        print(f"-- {lab}: lines {k}..{max(ends)}, {tot} instructions, VALU {sum(n for i, n in c.items() if i.startswith('v_'))}, "
              f"LDS {sum(n for i, n in c.items() if i.startswith('ds_'))}")
        print("   " + ", ".join(f"{i} {n}" for i, n in c.most_common(28)))


if __name__ == "__main__":
    main(*sys.argv[1:])
