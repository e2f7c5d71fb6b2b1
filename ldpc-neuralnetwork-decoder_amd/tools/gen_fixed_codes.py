#!/usr/bin/env python3
"""Generate csrc/gen/fixed_codes.hpp: compile-time schedules for the codes the reference ships.

The reference decodes exactly two codes (5G LDPC CODES/NR_2_0_4.txt and NR_2_0_32.txt, copied to
codes/).  For those, libldpc_amd carries a flooding kernel whose whole schedule -- which wave
updates which block-row and column, every LDS slot offset and circulant shift -- is a set of
compile-time constants, so the iteration loop is straight-line code with immediate LDS offsets
and no descriptor decoding.  Any other graph uses the table-driven kernel.

The slot numbering and the wave schedule are the ones graph.cpp computes at runtime (same LPT
rule, same tie-breaking), so both kernels hold identical LDS images.

    python tools/gen_fixed_codes.py   (run from ldpc-neuralnetwork-decoder_amd/; Makefile does it)
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CODES = [("BG2_Z4", os.path.join(ROOT, "codes", "NR_2_0_4.txt"), 4),
         ("BG2_Z32", os.path.join(ROOT, "codes", "NR_2_0_32.txt"), 32)]
W = 4


def load(path):
    with open(path) as f:
        return [[int(float(x)) for x in line.split()] for line in f if line.strip()]


def lpt(tasks, cost, w):
    order = sorted(range(len(tasks)), key=lambda i: -cost[i])  # stable for ties
    per = [[] for _ in range(w)]
    load_ = [0.0] * w
    for i in order:
        k = min(range(w), key=lambda j: load_[j])
        per[k].append(tasks[i])
        load_[k] += cost[i]
    return [sorted(p) for p in per]


def balance(tasks, cost, w):
    """LPT, then moves / swaps of single tasks between the heaviest wave and the others while the
    heaviest wave's load drops (the phase ends at a barrier: its time is the largest load)."""
    per = lpt(tasks, cost, w)
    c = dict(zip(tasks, cost))
    load = lambda p: sum(c[t] for t in p)
    improved = True
    while improved:
        improved = False
        per.sort(key=load, reverse=True)
        top = per[0]
        best = (load(top), None)
        for q in range(1, w):
            o = per[q]
            for t in top:  # move t from top to o
                m = max(load(top) - c[t], load(o) + c[t])
                if m < best[0] - 1e-9:
                    best = (m, ("move", t, q))
                for u in o:  # swap t and u
                    m = max(load(top) - c[t] + c[u], load(o) - c[u] + c[t])
                    if m < best[0] - 1e-9:
                        best = (m, ("swap", t, q, u))
        if best[1] is not None:
            kind = best[1][0]
            if kind == "move":
                _, t, q = best[1]
                top.remove(t)
                per[q].append(t)
            else:
                _, t, q, u = best[1]
                top.remove(t)
                per[q].remove(u)
                top.append(u)
                per[q].append(t)
            improved = True
    return [sorted(p) for p in per]


def arr(name, vals):
    vals = list(vals) or [0]
    body = ", ".join(str(v) for v in vals)
    return f"    static constexpr int {name}[{len(vals)}] = {{{body}}};\n"


def gen(name, base, z):
    mb, nb = len(base), len(base[0])
    blocks = [(r, c, base[r][c] % z) for r in range(mb) for c in range(nb) if base[r][c] >= 0]
    dv = [0] * nb
    dc = [0] * mb
    for r, c, _ in blocks:
        dv[c] += 1
        dc[r] += 1
    slot = []
    n = 0
    for r, c, _ in blocks:
        if dv[c] >= 2:
            slot.append(n)
            n += 1
        else:
            slot.append(-1)
    row_ptr = [0]
    for r in range(mb):
        row_ptr.append(row_ptr[-1] + dc[r])
    rows = list(range(mb))
    nslot = [sum(1 for i in range(row_ptr[r], row_ptr[r + 1]) if slot[i] >= 0) for r in rows]
    # per-iteration SIMD pipe cycles of one wave's share (tools/ubench costs at 4 waves / SIMD):
    # check row: the two minima (half-rate min / med3), sign parity, per slot edge compare +
    # select + sign, row constants; column: the exclusive ordered sums (full-rate adds) + its LDS
    # reads / writes issued
    rcost = [4.1 * n_min_ops(dc[r]) + 2.2 * (dc[r] // 2) + 10.4 * nslot[r] + 12 + 2.0 * dc[r] for r in rows]
    vcols = [c for c in range(nb) if dv[c] != 1]
    vcost = [1.94 * (dv[c] * (dv[c] - 1) // 2 + dv[c]) + 2.0 * dv[c] + 6 for c in vcols]
    chk = balance(rows, rcost, W)
    var = balance(vcols, vcost, W)
    bw = lpt(list(range(nb)), [1.0] * nb, W)
    col_blocks = [[i for i, b in enumerate(blocks) if b[1] == c] for c in range(nb)]
    col_ptr = [0]
    col_slot, col_shift = [], []
    for c in range(nb):
        for i in col_blocks[c]:
            col_slot.append(slot[i])
            col_shift.append(blocks[i][2])
        col_ptr.append(len(col_slot))

    def flat(lists):
        ptr = [0]
        out = []
        for l in lists:
            out += l
            ptr.append(len(out))
        return ptr, out

    cp, cl = flat(chk)
    vp, vl = flat(var)
    bp, bl = flat(bw)
    s = f"struct {name} {{\n"
    s += f"    static constexpr int Z = {z}, Mb = {mb}, Nb = {nb}, N = {nb * z}, NSLOTS = {n}, W = {W};\n"
    s += f"    static constexpr int NBLOCKS = {len(blocks)};\n"
    s += arr("BLK_ROW", [b[0] for b in blocks])
    s += arr("BLK_COL", [b[1] for b in blocks])
    s += arr("BLK_SHIFT", [b[2] for b in blocks])
    s += arr("ROW_PTR", row_ptr)
    s += arr("ROW_SLOT", slot)
    s += arr("ROW_COL", [b[1] for b in blocks])
    s += arr("ROW_SHIFT", [b[2] for b in blocks])
    s += arr("COL_PTR", col_ptr)
    s += arr("COL_SLOT", col_slot)
    s += arr("COL_SHIFT", col_shift)
    s += arr("CHK_PTR", cp)
    s += arr("CHK_ROWS", cl)
    s += arr("VAR_PTR", vp)
    s += arr("VAR_COLS", vl)
    s += arr("BW_PTR", bp)
    s += arr("BW_COLS", bl)
    s += task_schedule(blocks, slot, dc, dv, row_ptr, col_blocks, z)
    # one frame per lane, 6 waves (flood_w6.inc): the fixed kernel's slot numbering
    s += task_schedule(blocks, slot, dc, dv, row_ptr, col_blocks, z, W=6, prefix="S", frames=1, add=1.94,
                       remap=False)
    s += "};\n\n"
    return s


# ---- frame-pair kernel (flood.hip flood_pair_kernel): 8 waves, each lane carries two frames
PW = 8


def n_min_ops(d):
    """half-rate min / med3 ops for the two smallest of d magnitudes (flood.hip two_smallest)"""
    if d <= 1:
        return 0
    if d == 2:
        return 2
    return 2 + 5 * ((d - 3) // 3) + 2 * ((d - 3) % 3)


def var_task_adds(d, lo, hi):
    """v_pk_add_f32 of a column task writing outputs [lo, hi): the prefix P_1..P_{hi-1} (P_d, the
    APP, when hi == d) and the tails sum_{e in [lo, hi)} (d - 1 - e)"""
    pre = d if hi == d else hi - 1
    return pre + sum(d - 1 - e for e in range(lo, hi))


def var_task_cost(d, lo, hi, add=2.6):
    # pipe cycles at 4 waves / SIMD (tools/ubench): v_pk_add_f32 2.6 (the pair kernel), v_add_f32
    # 1.94 (one frame per lane); + LDS reads / writes issued
    return add * var_task_adds(d, lo, hi) + 1.0 * d + 1.5 * (hi - lo) + 6.0


def split_column(d, parts, add=2.6):
    """output ranges [lo, hi) of a degree-d column cut into `parts` tasks of about equal cost"""
    bounds = [0]
    for q in range(1, parts):
        # the cut after which the first q parts hold q/parts of the cost (greedy on prefix cost)
        total = var_task_cost(d, 0, d, add)
        best = min(range(bounds[-1] + 1, d), key=lambda h: abs(
            sum(var_task_cost(d, bounds[i], bounds[i + 1], add) for i in range(len(bounds) - 1))
            + var_task_cost(d, bounds[-1], h, add) - q * total / parts))
        bounds.append(best)
    bounds.append(d)
    return [(bounds[i], bounds[i + 1]) for i in range(parts)]


def row_cost(dcr, nslot, frames=2):
    # per frame: the two minima (half rate, 4.1), sign parity (bitop3 per two messages), per slot
    # edge compare + select + sign (4.1 + 4.1 + 2.2), row constants; x frames per lane
    return frames * (4.1 * n_min_ops(dcr) + 2.2 * (dcr // 2) + 10.4 * nslot + 12.0) + 2.0 * dcr


def makespan(tasks, cost, w):
    per = lpt(tasks, cost, w)
    loads = [sum(cost[tasks.index(t)] for t in p) for p in per]
    return max(loads), per


def task_schedule(blocks, slot, dc, dv, row_ptr, col_blocks, z, W=PW, prefix="P", frames=2, add=2.6,
                  remap=True):
    """Rows (LPT + refinement) and variable tasks (columns split by output range while that lowers
    the LPT makespan) for W waves.  frames / add: lanes' frames and the pipe cost of one ordered
    add (2 frames on v_pk_add_f32, or 1 on v_add_f32)."""
    mb = len(dc)
    nb = len(dv)
    # rows
    rows = list(range(mb))
    rc = [row_cost(dc[r], sum(1 for i in range(row_ptr[r], row_ptr[r + 1]) if slot[i] >= 0), frames) for r in rows]
    chk = balance(rows, rc, W)
    # variable tasks: split the heaviest columns while the LPT makespan improves
    vcols = [c for c in range(nb) if dv[c] >= 2]
    parts = {c: 1 for c in vcols}

    def tasks_of(parts):
        t = []
        for c in vcols:
            for lo, hi in split_column(dv[c], parts[c], add):
                t.append((c, lo, hi))
        return t

    def span(parts):
        t = tasks_of(parts)
        cost = [var_task_cost(dv[c], lo, hi, add) for c, lo, hi in t]
        per = balance(t, cost, W)
        c = dict(zip(t, cost))
        return max(sum(c[x] for x in p) for p in per), per

    best, per = span(parts)
    while True:
        t = tasks_of(parts)
        cost = [var_task_cost(dv[c], lo, hi, add) for c, lo, hi in t]
        heavy = t[max(range(len(t)), key=lambda i: cost[i])][0]
        trial = dict(parts)
        trial[heavy] += 1
        if trial[heavy] > dv[heavy]:
            break
        m, p2 = span(trial)
        if m >= best - 1e-9:
            break
        best, per, parts = m, p2, trial
    # slot numbering of the pair image: column-major, heaviest columns first, so the slots of the
    # waves with the most messages sit below the 64 KB reach of a ds_read's 16-bit offset
    order = sorted(vcols, key=lambda c: -dv[c])
    nslots = sum(1 for x in slot if x >= 0)
    pslot = [-1] * nslots
    n = 0
    for c in order:
        for i in col_blocks[c]:
            pslot[slot[i]] = n
            n += 1
    if not remap:
        pslot = list(range(nslots))
    vt_ptr, vt_col, vt_lo, vt_hi = [0], [], [], []
    for p in per:
        for c, lo, hi in sorted(p):
            vt_col.append(c)
            vt_lo.append(lo)
            vt_hi.append(hi)
        vt_ptr.append(len(vt_col))
    cp = [0]
    cl = []
    for p in chk:
        cl += p
        cp.append(len(cl))
    s = f"    // {prefix}: {W} waves, {frames} frame(s) per lane; variable tasks (column, outputs [lo, hi)); slot map\n"
    s += f"    static constexpr int {prefix}W = {W};\n"
    s += arr(f"{prefix}_CHK_PTR", cp)
    s += arr(f"{prefix}_CHK_ROWS", cl)
    s += arr(f"{prefix}_VT_PTR", vt_ptr)
    s += arr(f"{prefix}_VT_COL", vt_col)
    s += arr(f"{prefix}_VT_LO", vt_lo)
    s += arr(f"{prefix}_VT_HI", vt_hi)
    s += arr(f"{prefix}_SLOT", pslot)
    return s


def main(out):
    text = ("// GENERATED by tools/gen_fixed_codes.py from codes/NR_2_0_{4,32}.txt -- do not edit.\n"
            "// Compile-time flooding schedules for the two codes the reference ships (see that script).\n"
            "#pragma once\n\nnamespace ldpc {\nnamespace fixed {\n\n")
    for name, path, z in CODES:
        text += gen(name, load(path), z)
    text += "}  // namespace fixed\n}  // namespace ldpc\n"
    os.makedirs(os.path.dirname(out), exist_ok=True)
    old = open(out).read() if os.path.exists(out) else None
    if old != text:
        with open(out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "..", "csrc", "gen", "fixed_codes.hpp"))
