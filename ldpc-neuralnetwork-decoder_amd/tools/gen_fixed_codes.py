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
    chk = balance(rows, rcost, W)
    vt_pair = var_schedule(vcols, dv, W, pairs=True)
    vt_single = var_schedule(vcols, dv, W, pairs=False)
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
    for pre, sched in (("VT", vt_pair), ("VS", vt_single)):
        # per wave: the distinct columns of its tasks (LLRs, init, shifts), then the tasks
        # (column A, column B or -1, outputs [lo, hi)); VT pairs columns on v_pk_add_f32, VS does not
        vp, vl = flat([sorted({t[0] for t in p} | {t[1] for t in p if t[1] >= 0}) for p in sched])
        tp, tl = flat(sched)
        s += arr(f"{pre}_COL_PTR", vp)
        s += arr(f"{pre}_COLS", vl)
        s += arr(f"{pre}_PTR", tp)
        s += arr(f"{pre}_A", [t[0] for t in tl])
        s += arr(f"{pre}_B", [t[1] for t in tl])
        s += arr(f"{pre}_LO", [t[2] for t in tl])
        s += arr(f"{pre}_HI", [t[3] for t in tl])
    s += arr("BW_PTR", bp)
    s += arr("BW_COLS", bl)
    s += "};\n\n"
    return s


def n_min_ops(d):
    """half-rate min / med3 ops for the two smallest of d magnitudes (flood.hip two_smallest)"""
    if d <= 1:
        return 0
    if d == 2:
        return 2
    return 2 + 5 * ((d - 3) // 3) + 2 * ((d - 3) % 3)


def var_task_ops(DA, DB, lo, hi):
    """Instruction counts of a variable task (flood_dev.hpp FixedBody::task): outputs [lo, hi) of
    column A (degree DA) and, when DB > 0, of column B (degree DB <= DA) on v_pk_add_f32 pairs.
    Per output e: acc[e] = P_e, then + c_J for J = e + 1 .. D - 1 (the reference's ascending
    exclusive sum, traditional_decoders.py:235-250); prefix adds P_J -> P_{J+1} as far as an output
    or an APP (the column's last prefix) needs them.  Returns (pk adds, scalar adds, LDS reads,
    LDS writes, APPs)."""
    hasB = DB > 0 and lo < DB
    if not hasB:
        DB = 0
    nprefA = DA if hi == DA else max(hi - 1, 0)
    blast = hasB and lo <= DB - 1 < hi  # the task holding B's last output also takes B's APP
    npref = max(nprefA, DB if blast else 0)
    pk = sc = 0
    for J in range(DA):
        for e in range(lo, min(J, hi)):
            if J < DB:
                pk += 1
            else:
                sc += 1
        if J < npref:
            if J < DB:
                pk += 1
            else:
                sc += 1
    writes = (hi - lo) + (max(0, min(hi, DB) - lo) if hasB else 0)
    return pk, sc, DA + DB, writes, int(hi == DA) + int(blast)


def var_task_cost(DA, DB, lo, hi):
    """Cycles of a variable task inside the running kernel: least squares over the measured phase
    times of both schedules (tools/flood_timeline.py on the timeline builds, profiles/r04_flood_timeline_*):
    8.2 per v_pk_add_f32 (its dependent chains issue slower than the 2.6-cycle ubench rate), 4.85
    per v_add_f32, 18.1 per LDS read or write, 33.6 per task."""
    pk, sc, rd, wr, apps = var_task_ops(DA, DB, lo, hi)
    return 8.21 * pk + 4.85 * sc + 18.12 * (rd + wr) + 33.6


def var_schedule(vcols, dv, w, pairs=True):
    """Variable tasks per wave.  Columns sorted by degree; every pattern of pairing neighbours in
    that order (pairs=True; a pair's exclusive sums share v_pk_add_f32 instructions, the smaller
    column's adds riding along for free), each balanced over the waves (LPT + move / swap
    refinement); the smallest makespan wins (ties: least total cost).  A column is never split by
    output range over two waves: every output reads all of the column's messages and is written in
    place, so a split column's writes would race the other wave's reads within the phase.
    Returns [[(A, B or -1, 0, degree of A)]] per wave."""
    cols = sorted(vcols, key=lambda c: (-dv[c], c))
    n = len(cols)
    patterns = [[]]
    if pairs:
        def pats(i):
            if i >= n:
                return [[]]
            out = [[(cols[i],)] + p for p in pats(i + 1)]
            if i + 1 < n:
                out += [[(cols[i], cols[i + 1])] + p for p in pats(i + 2)]
            return out
        patterns = pats(0)
    else:
        patterns = [[(c,) for c in cols]]
    best = None
    for pat in patterns:
        t = [(u[0], u[1] if len(u) > 1 else -1, 0, dv[u[0]]) for u in pat]
        cost = [var_task_cost(dv[a], dv[b] if b >= 0 else 0, lo, hi) for a, b, lo, hi in t]
        per = balance(t, cost, w)
        c = dict(zip(t, cost))
        cur = (max(sum(c[x] for x in p) for p in per), sum(cost), per)
        key = (round(cur[0], 6), cur[1])
        if best is None or key < best[0]:
            best = (key, cur[2])
    return [sorted(p) for p in best[1]]


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
