#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 SQLite database (rocpd format, rocprofv3 -d DIR -o NAME).

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db [out.csv]

Prints (and optionally writes as CSV) Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs,
MaxNs in the layout of rocprofv3's --stats kernel_stats.csv, from the `kernels` view.
"""
import csv
import sqlite3
import sys


def stats(db):
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = con.execute(f"select {name}, count(*), sum(end - start), min(end - start), max(end - start) "
                       f"from kernels group by {name} order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [{"Name": r[0], "Calls": r[1], "TotalDurationNs": r[2], "AverageNs": r[2] / r[1],
             "Percentage": 100.0 * r[2] / tot, "MinNs": r[3], "MaxNs": r[4]} for r in rows]


def main(db, out=None):
    st = stats(db)
    for r in st[:20]:
        print(f"{r['Name'][:90]:90s} {r['Calls']:6d} avg {r['AverageNs'] / 1e3:10.1f} us {r['Percentage']:6.2f}%")
    if out:
        with open(out, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(st[0].keys()))
            w.writeheader()
            w.writerows(st)


if __name__ == "__main__":
    main(*sys.argv[1:])
