"""Per-rank compute of the sharded C5 build at N ranks, measured on one GPU (the driver's 8-GPU
node runs the real thing): the last line-aligned 1/N range is counted, parsed into global ids,
routed to N owners, and a row slice of the same entry count is built.  The RCCL all-to-all is
not in these numbers.  Usage: python tools/shard_probe.py [N] [steps]"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import torch

    import bench
    from gfa2network_amd import synth
    from gfa2network_amd.shard import HipEngine

    n_ranks = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    wl = synth.WORKLOADS["C5"]
    dev = synth.DeviceInput(wl.n_segments, wl.n_links, seed=0, rc_tag=wl.rc_tag, device=0)
    # the last range (L lines only: the generator writes every S line first)
    lo = bench._line_start_device(dev.ptr, dev.len, (n_ranks - 1) * dev.len // n_ranks)
    hi = dev.len
    buf = bench._DevBytes(dev.ptr + lo, hi - lo)
    eng = HipEngine(0)
    opts = dict(directed=False, bidirected=False, weight_tag=None, dtype="float64")
    n_global = wl.n_segments
    out = {"n_ranks": n_ranks, "range_bytes": hi - lo}
    tm = {"count": [], "build": [], "route": [], "csr": []}
    for it in range(steps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cnt = eng.count(buf)
        t1 = time.perf_counter()
        local = eng.build_decimal(buf, opts, n_global - cnt[1], n_global, view=True)  # S lines precede it
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rr, cc, _, st = eng.route_triplets(local.rows, local.cols, None, "float64", None, n_global, n_ranks, False)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        # a slice of the same entry count: this range's triplets as rows [0, n_global / N * N) ... all rows
        eng.csr_pair((rr, cc, None), None, False, 0, n_global, n_global, "float64", True, -1)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        if it:
            for k, v in zip(tm, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
                tm[k].append(v * 1e3)
    out.update({k: round(sum(v) / len(v), 3) for k, v in tm.items()})
    out["entries"] = int(local.rows.numel())
    out["counts"] = cnt
    out["a2a_bytes_out"] = int(local.rows.numel()) * 8 * (n_ranks - 1) // n_ranks
    print(json.dumps(out))
    eng.close()
    dev.free()


if __name__ == "__main__":
    main()
