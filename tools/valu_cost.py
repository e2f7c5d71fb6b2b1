#!/usr/bin/env python3
"""Static VALU pipe-cycle count of a kernel's hot blocks, with the issue costs measured on MI355X
by tools/ubench/valu_banks (profiles/r02_ubench_valu_banks.jsonl, one workgroup of 4 waves per SIMD):
    2 cycles per wave64 instruction: v_add_f32, v_xor_b32, v_bitop3_b32 with VGPR operands, ...
    4 cycles: v_min/v_max/v_med3_f32, v_cmp_*, v_cndmask_b32, v_bfi_b32, v_exp/v_log/v_rcp, and any
              VALU op with an SGPR source (literal and inline constants are full rate)
    ~2.5 cycles: v_pk_add_f32 (two adds)
usage: valu_cost.py <kernel.s> [min-instructions-per-block | --hot]
(kernel.s: hipcc -S --cuda-device-only of a file that includes csrc/flood.hip with
LDPC_FLOOD_KERNELS_ONLY and instantiates flood_fixed_kernel<BG2_Z32, MINSUM, ES_OFF> alone)
"""
import re
import sys

HALF = ("v_min_", "v_max_", "v_med3_", "v_cmp_", "v_cndmask_", "v_bfi_", "v_readfirstlane", "v_readlane", "v_writelane",
        "v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_")  # transcendentals: 4 at 4 waves/SIMD (8 alone)


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


def hot_loop_weight(path):
    """Issue-cost weight of the flood kernel's hot iteration (fast check phase + variable phase of
    every wave): modelled VALU pipe cycles / (2 x VALU instructions).  Blocks: >= 250 instructions
    and >= 40 LDS ops (the per-iteration phases; the slow MinSumStats blocks have > 600 half-rate
    ops and the decision-taking last-iteration blocks < 40 LDS ops)."""
    blocks = parse(path)
    sel = []
    for name, ins in blocks:
        v = [i for i in ins if i.startswith("v_")]
        half = sum(1 for i in v if cost(i) == 4.0)
        lds = sum(1 for i in ins if i.startswith("ds_"))
        if len(ins) >= 250 and lds >= 40 and half < 600:
            sel.append((name, len(v), sum(cost(i) for i in v)))
    nv = sum(s[1] for s in sel)
    cyc = sum(s[2] for s in sel)
    return {"blocks": [s[0] for s in sel], "valu_instructions": nv, "valu_cycles": cyc, "weight": cyc / (2.0 * nv)}


def parse(path):
    lines = open(path).read().split("\n")
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
    return blocks


def main():
    if len(sys.argv) > 2 and sys.argv[2] == "--hot":
        import json
        print(json.dumps(hot_loop_weight(sys.argv[1]), indent=1))
        return
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
