#!/usr/bin/env python3
"""Instruction mix of one kernel in a device assembly file (hipcc --cuda-device-only -S).

    python tools/isa_stats.py <file.s> <symbol-substring> [top]

Prints the static instruction counts (whole kernel), the VGPR / SGPR / spill figures of the
kernel's metadata, and the counts inside the largest loop body (the iteration loop of the flood
kernels: the block between the most-instructions back-edge label and its branch).
"""
import collections
import re
import sys


def kernel_body(text, sub):
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n", text, re.M):
        if sub in m.group(1):
            end = text.find(".Lfunc_end", m.end())
            return m.group(1), text[m.end():end]
    raise SystemExit(f"no kernel matching {sub}")


def meta(text, name):
    i = text.find(f".name:           {name}")
    if i < 0:
        return {}
    blk = text[max(0, i - 3000):i + 3000]
    out = {}
    for k in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count", "agpr_count"):
        m = re.search(rf"\.{k}:\s+(\d+)", blk)
        if m:
            out[k] = int(m.group(1))
    return out


def main(path, sub, top=30):
    text = open(path).read()
    name, body = kernel_body(text, sub)
    lines = body.split("\n")
    ins = [l.split()[0] for l in lines if l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;")]
    c = collections.Counter(ins)
    print(name)
    print("meta", meta(text, name))
    nv = sum(n for k, n in c.items() if k.startswith("v_"))
    print(f"static: {len(ins)} instructions, VALU {nv}, LDS {sum(n for k, n in c.items() if k.startswith('ds_'))}, "
          f"SALU {sum(n for k, n in c.items() if k.startswith('s_'))}")
    for k, n in c.most_common(int(top)):
        print(f"  {n:6d} {k}")


if __name__ == "__main__":
    main(*sys.argv[1:])
