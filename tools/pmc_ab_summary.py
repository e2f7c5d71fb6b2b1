#!/usr/bin/env python3
"""Per-kernel sums of the SQ passes written by tools/gpu_pmc_ab.sh.
    python tools/pmc_ab_summary.py gpurun_out/pmcab_<TAG> [kernel substring]"""
import collections
import csv
import os
import sys


def short(name):
    return name.replace("ldpc::(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def main(d, sub="mlp"):
    for lib in sorted(os.listdir(d)):
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for p in ("p1", "p2", "p3", "p4"):
            f = os.path.join(d, lib, p, "run_counter_collection.csv")
            if not os.path.exists(f):
                for root, _, files in os.walk(os.path.join(d, lib, p)):
                    for n in files:
                        if n.endswith("counter_collection.csv"):
                            f = os.path.join(root, n)
            if not os.path.exists(f):
                continue
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                if sub not in k:
                    continue
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((p, r.get("Dispatch_Id", "")))
        for k, c in agg.items():
            wc = c.get("SQ_WAVE_CYCLES", 0) or 1
            n = max(1, len([x for x in disp[k] if x[0] == "p1"]))
            print(f"{lib:10s} {k[:48]:48s} launches {n}")
            print(f"    wait_any {c.get('SQ_WAIT_ANY', 0) / wc:.3f}  wait_inst {c.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}"
                  f"  active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f}  valu_active {c.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}"
                  f"  wait_lds {c.get('SQ_WAIT_INST_LDS', 0) / wc:.3f}")
            busy = c.get("SQ_BUSY_CYCLES", 0)
            gui = c.get("GRBM_GUI_ACTIVE", 0)
            print(f"    mfma_busy_cycles/launch {c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / n:.4g}  grbm_gui/launch {gui / n:.4g}"
                  f"  sq_busy/launch {busy / n:.4g}  waves {c.get('SQ_WAVES', 0) / n:.4g}")
            print(f"    per launch: VALU {c.get('SQ_INSTS_VALU', 0) / n:.4g}  LDS {c.get('SQ_INSTS_LDS', 0) / n:.4g}"
                  f"  VMEM {c.get('SQ_INSTS_VMEM', 0) / n:.4g}  LDS bank conflict {c.get('SQ_LDS_BANK_CONFLICT', 0) / n:.4g}"
                  f"  active_lds {c.get('SQ_ACTIVE_INST_LDS', 0) / n:.4g}  SALU {c.get('SQ_INSTS_SALU', 0) / n:.4g}")
            if "FETCH_SIZE" in c:  # MI355X_MICROARCH.md HBM section: bytes = 2 FETCH_SIZE KB + WRITE_SIZE KB
                print(f"    per launch: read {2 * c['FETCH_SIZE'] * 1024 / n / 1e6:.1f} MB  write {c.get('WRITE_SIZE', 0) * 1024 / n / 1e6:.1f} MB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "mlp")
