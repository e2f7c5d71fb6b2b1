#!/usr/bin/env python3
"""Per-wave, per-phase timeline of the flooding decoder (timeline build, tools/build_timeline.sh).

    LDPC_AMD_LIB=.../variants/timeline.so LDPC_TIMELINE_OUT=tl.bin python bench.py --steps 1 ...
    python tools/flood_timeline.py tl.bin [out.json]

The dump holds, for the first kTlWgs workgroups x 4 waves, s_memtime (shader clock) stamps:
[0] after the init barrier, then per iteration it: [1+4it] check phase done, [2+4it] barrier 1
passed, [3+4it] variable phase done, [4+4it] barrier 2 passed.  Reported per wave index (the
fixed kernel specialises its work per wave):
  * check / var: cycles from the previous barrier to the end of the wave's own phase work
  * wait1 / wait2: cycles the wave then waits at the barrier
  * critical: how often the wave is the last to reach the barrier (the one the others wait on)
averaged over the recorded workgroups and the iterations 1 .. max_iter - 2 (the first carries the
prologue, the last takes decisions).
"""
import json
import sys

import numpy as np


def main(path, out=None):
    with open(path, "rb") as f:
        hdr = np.frombuffer(f.read(16), dtype=np.int32)
        nwg, nw, per, max_iter = (int(x) for x in hdr)
        t = np.frombuffer(f.read(), dtype=np.uint64).astype(np.int64).reshape(nwg, nw, per)
    t = t[(t[:, :, 0] > 0).all(axis=1)]  # recorded workgroups only
    its = range(1, max(2, max_iter - 1))
    rows = {k: [] for k in ("check", "wait1", "var", "wait2")}
    crit1, crit2 = np.zeros(nw), np.zeros(nw)
    iter_cycles = []
    for it in its:
        b = 4 * it
        start = t[:, :, b]  # barrier 2 of the previous iteration passed (or init)
        ce, b1, ve, b2 = (t[:, :, b + k] for k in (1, 2, 3, 4))
        rows["check"].append((ce - start).mean(axis=0))
        rows["wait1"].append((b1 - ce).mean(axis=0))
        rows["var"].append((ve - b1).mean(axis=0))
        rows["wait2"].append((b2 - ve).mean(axis=0))
        crit1 += np.bincount(np.argmax(ce, axis=1), minlength=nw)
        crit2 += np.bincount(np.argmax(ve, axis=1), minlength=nw)
        iter_cycles.append((b2.max(axis=1) - start.min(axis=1)).mean())
    res = {"workgroups": int(t.shape[0]), "waves": nw, "iterations_used": list(its),
           "cycles_per_iteration": float(np.mean(iter_cycles))}
    for k, v in rows.items():
        res[k] = [round(float(x), 1) for x in np.mean(v, axis=0)]
    n = crit1.sum()
    res["critical_check"] = [round(float(x) / n, 3) for x in crit1]
    res["critical_var"] = [round(float(x) / n, 3) for x in crit2]
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
