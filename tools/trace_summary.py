#!/usr/bin/env python3
"""Per-kernel duration summary of a rocprofv3 --kernel-trace CSV (median/min/max, us).

    python tools/trace_summary.py <dir-with-run_kernel_trace.csv> [frames]
"""
import collections
import csv
import glob
import re
import sys


def main(d, frames=None):
    f = glob.glob(f"{d}/**/run_kernel_trace.csv", recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        m = re.search(r"((?:gnn|flood|bf16|qpsk|count|batch|train|csr|gather|residual|output_layer)\w*(<[^>]*>)?)", n)
        agg[m.group(1) if m else n[:40]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for n, v in sorted(agg.items(), key=lambda x: -sum(x[1]))[:10]:
        v = sorted(v)
        med = v[len(v) // 2]
        extra = f" {med * 1e3 / float(frames):8.1f} ns/frame" if frames else ""
        print(f"{n[:52]:52s} n={len(v):4d} med={med:9.1f} min={v[0]:9.1f} max={v[-1]:9.1f}{extra}")


if __name__ == "__main__":
    main(*sys.argv[1:])
