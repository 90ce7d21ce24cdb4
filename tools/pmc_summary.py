#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports
exactly 1/2 of the bytes of a wide coalesced streaming read, so the prescribed figure is
traffic = 2 x FETCH_SIZE + WRITE_SIZE.  We check that calibration on this pipeline's own
pure-streaming kernel (k_tile_count reads the input once: FETCH_SIZE x 2 must equal the input
size) and record it.  Kernels that mix streaming and random 32-64 B accesses are
uncalibrated: the raw FETCH_SIZE (random 64-B requests counted once) is kept beside the
corrected figure.

usage: pmc_summary.py <pmc dir with FETCH_SIZE/ and WRITE_SIZE/> <input bytes> <out.json>
"""
import collections
import csv
import json
import sys
from pathlib import Path


def load(d: Path, counter: str):
    rows = list(csv.DictReader(open(d / counter / "run_counter_collection.csv")))
    agg = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[name].append(float(r["Counter_Value"]) * 1024.0)  # KiB -> bytes
    return agg


def main():
    d, in_bytes, out = Path(sys.argv[1]), int(sys.argv[2]), Path(sys.argv[3])
    fetch, write = load(d, "FETCH_SIZE"), load(d, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [0.0])
        w = write.get(k, [0.0])
        fa, wa = sum(f) / len(f), sum(w) / len(w)
        kernels[k] = {"launches": len(f), "fetch_size_bytes_raw": round(fa), "write_size_bytes": round(wa),
                      "traffic_bytes_per_launch": round(2 * fa + wa)}
    cal = kernels.get("g2n::k_tile_count", {})
    doc = {
        "source": str(d),
        "correction": "traffic = 2*FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md §HBM, gfx950 FETCH_SIZE = 1/2 of "
                      "wide streaming reads)",
        "calibration": {"kernel": "g2n::k_tile_count (reads the input once + a 16-B halo per 32 KiB tile, coalesced 16 B/lane)",
                        "input_bytes": in_bytes, "fetch_size_x2": 2 * cal.get("fetch_size_bytes_raw", 0),
                        "ratio": round(2 * cal.get("fetch_size_bytes_raw", 0) / max(in_bytes, 1), 4)},
        "kernels": kernels,
    }
    out.write_text(json.dumps(doc, indent=1))
    print(json.dumps(doc["calibration"]))


if __name__ == "__main__":
    main()
