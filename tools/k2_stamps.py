"""Analyse the K2 (k_tile_parse<true>) phase stamps of a -DG2N_K2_STAMPS build.

usage: python tools/k2_stamps.py stamps.bin [out.json] [f1]
(f1: the bucket-finish stamps of a -DG2N_F1_STAMPS build: 0 entry, 1 loaded + counted, 2 placed,
3 rows sorted, 4 merged + offsets, 5 staged, 6 end; 9 = hardware id)
stamps.bin: n_tiles x 10 u64 — wall clock (100 MHz) at: 0 entry, 1 staged, 2 chunk masks,
3 chunk-rank scan, 4 start list, 5 kinds + line prefixes, 6 thread 0's lines parsed, 7 all lines
parsed (barrier), 8 end; 9 = XCC id << 32 | HW_ID.
Prints per-segment mean / median block time, the kernel span, the average number of blocks
resident per CU over the span, and the idle time between consecutive blocks on a CU.
"""
import json
import sys

import numpy as np

NAMES = ["stage", "masks", "scan", "starts", "classify", "parse_t0", "parse_all", "finish"]
TICK_NS = 10.0  # wall_clock64 at 100 MHz


LEAN_NAMES = ["stage_masks", "classify", "scan", "records", "parse", "finish"]
F1_NAMES = ["load_count", "place", "sort", "merge_scan", "stage", "write"]


def main():
    a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 10)
    a = a[a[:, 0] != 0]  # tiles that returned before the first stamp (the hash passes skip some)
    lean = bool((a[:, 7] == 0).all())  # k_tile_lean stamps 0..6 (and the hardware id in 9)
    names = LEAN_NAMES if lean else NAMES
    last = 6 if lean else 8
    if len(sys.argv) > 3 and sys.argv[3] == "f1":
        names, last = F1_NAMES, 6
    t = a[:, :last + 1].astype(np.int64)
    hw = a[:, 9]
    n = len(t)
    seg = np.diff(t, axis=1) * TICK_NS / 1e3  # us
    out = {"tiles": n}
    for k, name in enumerate(names):
        out[name] = {"mean_us": round(float(seg[:, k].mean()), 3), "median_us": round(float(np.median(seg[:, k])), 3),
                     "p90_us": round(float(np.percentile(seg[:, k], 90)), 3)}
    dur = (t[:, last] - t[:, 0]) * TICK_NS / 1e3
    span = (t[:, last].max() - t[:, 0].min()) * TICK_NS / 1e3
    out["block_us"] = {"mean": round(float(dur.mean()), 3), "median": round(float(np.median(dur)), 3)}
    out["span_us"] = round(float(span), 1)
    # CU identity: XCC, SE, SH, CU (HW_ID: CU_ID 8..11, SH_ID 12, SE_ID 13..15 on gfx9)
    xcc = (hw >> 32) & 0xF
    hwid = hw & 0xFFFFFFFF
    cu = (hwid >> 8) & 0xF
    sh = (hwid >> 12) & 0x1
    se = (hwid >> 13) & 0x7
    key = (xcc << 8) | (se << 5) | (sh << 4) | cu
    cus = np.unique(key)
    out["cus_seen"] = int(len(cus))
    out["avg_resident_blocks_per_cu"] = round(float(dur.sum() / (span * len(cus))), 3)
    gaps = []
    for c in cus:
        idx = np.flatnonzero(key == c)
        ends = np.sort(t[idx, last])
        starts = np.sort(t[idx, 0])
        # time in the span when this CU had no block resident
        ev = np.concatenate([np.stack([starts, np.ones_like(starts)], 1), np.stack([ends, -np.ones_like(ends)], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        live, prev, idle = 0, ev[0, 0], 0
        for x, d in ev:
            if live == 0:
                idle += x - prev
            live += d
            prev = x
        gaps.append(idle * TICK_NS / 1e3)
    out["cu_idle_us_mean"] = round(float(np.mean(gaps)), 2)
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2 and sys.argv[2] != "-":
        with open(sys.argv[2], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
