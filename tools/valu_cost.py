#!/usr/bin/env python3
"""Static VALU pipe-cycle count of a kernel's hot blocks, with the issue costs measured on MI355X
by tools/ubench/valu_banks (profiles/r02_ubench_valu_banks.jsonl, one workgroup of 4 waves per SIMD):
    2 cycles per wave64 instruction: v_add_f32, v_xor_b32, v_bitop3_b32 with VGPR operands, ...
    4 cycles: v_min/v_max/v_med3_f32, v_cmp_*, v_cndmask_b32, and any VALU op with an SGPR source
    ~2.5 cycles: v_pk_add_f32 (two adds)
usage: valu_cost.py <kernel.s> [min-instructions-per-block]
"""
import re
import sys

HALF = ("v_min_", "v_max_", "v_med3_", "v_cmp_", "v_cndmask_", "v_readfirstlane", "v_readlane", "v_writelane")


def cost(ins):
    op = ins.split()[0]
    if not op.startswith("v_"):
        return 0.0
    if op.startswith("v_pk_add_f32") or op.startswith("v_pk_mul_f32") or op.startswith("v_pk_fma_f32"):
        return 2.5
    if op.startswith(HALF):
        return 4.0
    srcs = ins.split(None, 1)[1].split(",")[1:] if " " in ins else []
    if any(re.match(r"\s*-?\|?s(\d+|\[)", s) for s in srcs):
        return 4.0
    return 2.0


def main():
    lines = open(sys.argv[1]).read().split("\n")
    thr = int(sys.argv[2]) if len(sys.argv) > 2 else 250
    blocks, cur = [], None
    for l in lines:
        m = re.match(r"^(\.LBB\S+|; %bb\.\d+):", l)
        if m:
            cur = [m.group(1), []]
            blocks.append(cur)
            continue
        if cur is not None:
            t = l.strip()
            if t and not t.startswith((".", ";")):
                cur[1].append(t)
    for name, ins in blocks:
        if len(ins) < thr:
            continue
        v = [i for i in ins if i.startswith("v_")]
        cyc = sum(cost(i) for i in v)
        half = sum(1 for i in v if cost(i) == 4.0)
        print(f"{name:12s} instr {len(ins):4d} valu {len(v):4d} half-rate {half:4d} pk {sum(1 for i in v if i.startswith('v_pk_')):4d} "
              f"lds {sum(1 for i in ins if i.startswith('ds_')):3d} valu_cycles {cyc:7.1f}")


if __name__ == "__main__":
    main()
