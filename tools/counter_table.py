#!/usr/bin/env python3
"""Per-kernel table from gpu_counters.sh passes: median duration, HBM bytes (2*FETCH_SIZE + WRITE_SIZE,
MI355X_MICROARCH.md gfx950 correction: FETCH_SIZE reports half of a wide streaming read), SQ
instruction mix and wait fractions, all per launch.

usage: counter_table.py <gpu_counters dir> [out.json commit]   (out.json: the summary bench.py reads)"""
import collections
import csv
import json
import sys
from pathlib import Path

d = Path(sys.argv[1])
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for p in sorted(d.glob("p*/")):
    for f in p.glob("run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[k][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for f in p.glob("run_kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
out = {}
for k, m in vals.items():
    per = collections.defaultdict(list)
    for (disp, cn), v in m.items():
        per[cn].append(sum(v))  # summed over dimensions (XCDs / SEs) of one dispatch
    avg = {cn: sum(v) / len(v) for cn, v in per.items()}
    row = {"ms": round(sorted(dur[k])[len(dur[k]) // 2], 3) if dur[k] else None,
           "launches": max(len({disp for (disp, cn) in m if cn == c}) for c in {cn for (_, cn) in m})}
    if "FETCH_SIZE" in avg:  # KiB
        row["traffic_bytes_per_launch"] = round((2 * avg["FETCH_SIZE"] + avg.get("WRITE_SIZE", 0)) * 1024)
        row["hbm_GB"] = round((2 * avg["FETCH_SIZE"] + avg.get("WRITE_SIZE", 0)) * 1024 / 1e9, 3)
        row["fetchx2_GB"] = round(2 * avg["FETCH_SIZE"] * 1024 / 1e9, 3)
        row["write_GB"] = round(avg.get("WRITE_SIZE", 0) * 1024 / 1e9, 3)
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        for cn in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if cn in avg:
                row[cn.replace("SQ_", "").lower() + "_frac"] = round(avg[cn] / wc, 3)
    for cn in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
               "SQ_LDS_BANK_CONFLICT", "SQ_BUSY_CYCLES"):
        if cn in avg:
            row[cn.replace("SQ_", "").lower()] = int(avg[cn])
    out[k] = row
for k, r in sorted(out.items(), key=lambda kv: -(kv[1]["ms"] or 0)):
    print(k[:40], json.dumps(r))
(d / "table.json").write_text(json.dumps(out, indent=1))
if len(sys.argv) > 3:
    Path(sys.argv[2]).write_text(json.dumps({
        "commit": sys.argv[3], "source": "tools/gpu_counters.sh (rocprofv3 --pmc, one pass per counter group, "
        "kernel-trace only) on `bench.py --steps 1 --warmup 0` (one build; launches = dispatches of the kernel "
        "in one pass)",
        "correction": "traffic = 2 * FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md: gfx950 FETCH_SIZE = 1/2 of a "
        "wide streaming read; WRITE_SIZE exact)", "kernels": out}, indent=1))
