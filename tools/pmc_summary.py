#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (tools/gpu_profile.sh output) into profiles/<tag>_pmc_<w>.json.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE on gfx950 reads exactly half
the bytes of a wide coalesced streaming read, so bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
(the counters are in KB).  Here the doubling is checked against a known byte count: the LLR
input of the flood decoder is B*N*4 bytes and it is read exactly once.

    python tools/pmc_summary.py gpurun_out/prof_<tag>_<w> <kernel-substring> <out.json> [expected_read_bytes|-] [per-call-kernel]
"""
import collections
import csv
import json
import os
import sys


def main(d, kern, out, expected_read=None, per_call=None):
    """per_call: a kernel-name substring launched once per call (e.g. once per GNN forward); when
    given, counters are summed over every kernel matching `kern` and divided by the number of
    such calls, so "per launch" means per call of a multi-kernel path."""
    agg = collections.defaultdict(list)
    calls = collections.Counter()
    for sub in sorted(os.listdir(d)):
        f = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        seen = set()
        for r in csv.DictReader(open(f)):
            if per_call and per_call in r["Kernel_Name"]:
                key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
                if key not in seen:
                    seen.add(key)
                    calls[r["Counter_Name"]] += 1
            if any(k in r["Kernel_Name"] for k in kern.split("|")):  # '|' separates alternatives
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    if per_call:
        res = {k: sum(v) / max(calls[k], 1) for k, v in agg.items()}
    else:
        res = {k: sum(v) / len(v) for k, v in agg.items()}
    waves = res.get("SQ_WAVES")
    out_d = {"kernel_substring": kern, "counters_per_launch": res}
    # the library build these counters describe (tools/gpu_profile.sh writes the sha256 of the .so
    # the profiled runs loaded); bench.py reports PMC-derived figures only for that same build
    stamp = os.path.join(d, "lib_sha256.txt")
    if os.path.exists(stamp):
        out_d["lib_sha256"] = open(stamp).read().split()[0]
    cos = os.path.join(d, "code_objects_sha256.txt")
    if os.path.exists(cos):
        out_d["code_objects_sha256"] = open(cos).read().split()
    if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
        read_b = 2 * res["FETCH_SIZE"] * 1024
        write_b = res["WRITE_SIZE"] * 1024
        out_d.update({"read_bytes_per_launch": read_b, "write_bytes_per_launch": write_b,
                      "bytes_per_launch": read_b + write_b,
                      "correction": "FETCH_SIZE x2 (gfx950 half-count for wide streaming reads), KB->B"})
        if expected_read:
            out_d["expected_read_bytes"] = float(expected_read)
            out_d["read_vs_expected"] = read_b / float(expected_read)
    if waves:
        out_d["per_wave"] = {k: v / waves for k, v in res.items() if k.startswith("SQ_")}
    # Derived utilisations (MI355X: 256 CUs x 4 SIMDs; GRBM_GUI_ACTIVE is the sum over 8 XCDs).
    # A SIMD issues one wave64 VALU instruction per 2 cycles (MI355X_MICROARCH.md: "issues each
    # VALU instruction over 2 cycles"); SQ_ACTIVE_INST_VALU counts quad-cycles a wave spends
    # issuing VALU (4 cycles per instruction for one wave alone); SQ_LDS_IDX_ACTIVE counts LDS
    # array cycles summed over CUs.
    cyc = res.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc and not per_call:
        d = {"cycles_per_launch": cyc}
        if "SQ_INSTS_VALU" in res:
            d["valu_pipe_frac"] = res["SQ_INSTS_VALU"] * 2 / (1024 * cyc)
        if "SQ_ACTIVE_INST_VALU" in res:
            d["valu_wave_active_frac"] = res["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * cyc)
        if "SQ_LDS_IDX_ACTIVE" in res:
            d["lds_busy_frac"] = res["SQ_LDS_IDX_ACTIVE"] / (256 * cyc)
        if "SQ_INST_CYCLES_SALU" in res:
            d["salu_busy_frac"] = res["SQ_INST_CYCLES_SALU"] * 4 / (1024 * cyc)
        if "SQ_WAVE_CYCLES" in res:
            d["waves_resident_per_simd"] = res["SQ_WAVE_CYCLES"] * 4 / (1024 * cyc)
        if "SQ_WAIT_ANY" in res and "SQ_ACTIVE_INST_ANY" in res:
            d["wait_over_issue"] = res["SQ_WAIT_ANY"] / res["SQ_ACTIVE_INST_ANY"]
        out_d["derived"] = d
    json.dump(out_d, open(out, "w"), indent=1)
    print(json.dumps(out_d, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    if len(a) > 3 and a[3] == "-":
        a[3] = None
    main(*a)
