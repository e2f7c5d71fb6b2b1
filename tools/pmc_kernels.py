#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 PMC passes (tools/gpu_profile.sh output directory):
HBM bytes per launch from FETCH_SIZE / WRITE_SIZE (MI355X_MICROARCH.md HBM section: gfx950
FETCH_SIZE counts half of a wide read: bytes = 2 FETCH_SIZE KB + WRITE_SIZE KB) and the SQ counters.

    python tools/pmc_kernels.py gpurun_out/prof_<tag>_<workload> [substring]
"""
import collections
import csv
import os
import sys


def short(name):
    n = name.replace("ldpc::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def main(d, sub="gnn"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(int))
    for p in sorted(os.listdir(d)):
        f = os.path.join(d, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k][r["Counter_Name"]] += 1
    out = {}
    for k in sorted(agg):
        if sub not in k:
            continue
        c = {n: agg[k][n] / cnt[k][n] for n in agg[k]}
        c["read_bytes"] = 2 * c.get("FETCH_SIZE", 0) * 1024
        c["write_bytes"] = c.get("WRITE_SIZE", 0) * 1024
        c["launches"] = cnt[k].get("FETCH_SIZE", 0)
        out[k] = c
        print(f"{k:40s} launches {c['launches']:4d}  read {c['read_bytes'] / 1e6:9.2f} MB  write "
              f"{c['write_bytes'] / 1e6:8.2f} MB  VALU {c.get('SQ_INSTS_VALU', 0):.3g}  LDS {c.get('SQ_INSTS_LDS', 0):.3g}")
    return out


if __name__ == "__main__":
    main(*sys.argv[1:])
