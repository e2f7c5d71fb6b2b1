#!/usr/bin/env python3
"""Per-stage kernel times of the wide-H GNN layer from a rocprofv3 kernel trace (tools/gpu_trace1s.sh):
each layer is gnn_wide_gm_kernel followed by five gnn_wgemm_kernel launches (projection v / c, GEMM1
v / c, GEMM2).   usage: python tools/wide_stages.py gpurun_out/tr1s_<tag>_<workload>"""
import collections
import csv
import os
import sys

rows = list(csv.DictReader(open(os.path.join(sys.argv[1], "run_kernel_trace.csv"))))
seq, cur = [], None
for r in rows:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "wide_gm" in n:
        cur = [d]
        seq.append(cur)
    elif "wgemm" in n and cur is not None:
        cur.append(d)
acc = collections.defaultdict(list)
for s in seq:
    for i, d in enumerate(s):
        acc[i].append(d)
names = ["group means", "projection v", "projection c", "GEMM1 v", "GEMM1 c", "GEMM2"]
for i in sorted(acc):
    print(f"{names[i] if i < len(names) else i:14s} {len(acc[i]):5d} launches {sum(acc[i]) / len(acc[i]):10.1f} us")
