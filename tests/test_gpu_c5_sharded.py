"""BASELINE config 5 as configured — ONE 16 GB file of 125M S / 500M L lines, ``directed=False``
(the undirected SUM CSR of convert_format(parse_gfa(...), "csr")) — byte-range-sharded over 8 ranks
(processes) on the box's one GPU, exchanging over gloo, against the same file built by one GPU
(VERDICT r05 item 1).

* decimal names ("1".."N", S lines first): the fast path (one-pass range parse into global ids, the
  evidence all-gather, triplets routed to row owners with one all-to-all-v);
* hashed names (unique, not decimal): the general owner protocol (names to owners, owner dedup,
  global first-touch ids, the id map back, the range's triplets remapped and routed).

The single-GPU build runs first in its own process and leaves only digests (xxh3-128 of indptr,
indices, data, the names blob and offsets; dtypes and shape), so its HBM is free before the ranks
start.  Each rank then preads only its line-aligned range (g2n_upload_file_range), builds its row
slice and sends it to rank 0 (gather_csr root=0; the names gathered to rank 0 as one blob), which
digests the gathered matrix the same way.  Bit for bit: the single-GPU build is pinned against the
oracle at C4 size (test_gpu_fullsize.py), this test pins the protocol at C5 size — the sizes where
all-to-all counts, slice offsets and the gathered index dtype would break first.  Per-rank stage
times and all-to-all bytes go to gpurun_out/c5_shard_<names>.json (copied to profiles/ by hand).
"""
import json
import os
import socket
import time

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(1100)]

N_S, N_L, WORLD, SEED = 125_000_000, 500_000_000, 8, 5
MODE = {"directed": False}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _digest(indptr, indices, data, blob, offs):
    import xxhash

    def h(a):
        a = np.ascontiguousarray(a)
        x = xxhash.xxh3_128()
        mv = memoryview(a.view(np.uint8).reshape(-1))
        for k in range(0, len(mv), 1 << 30):
            x.update(mv[k:k + (1 << 30)])
        return x.hexdigest()

    return {"indptr": [str(indptr.dtype), len(indptr), h(indptr)],
            "indices": [str(indices.dtype), len(indices), h(indices)],
            "data": [str(data.dtype), len(data), h(data)],
            "names_blob": [len(blob), h(blob)],
            "names_offsets": [len(offs), h(np.asarray(offs, dtype=np.int64))]}


def _one_gpu(rank, path, outdir):
    """The whole file on one GPU (its own process: the HBM is released when it exits)."""
    from gfa2network_amd import _native as nat

    t0 = time.perf_counter()
    raw = nat.build_from_path(path, nat.make_options(output=nat.OUT_CSR, want_node_names=True, **MODE))
    t_build = time.perf_counter() - t0
    assert raw.status == 0, raw.message
    d = _digest(raw.indptr, raw.indices, raw.data, raw.names_blob, raw.names_offsets)
    with open(os.path.join(outdir, "one_gpu.json"), "w") as fh:
        json.dump({"digest": d, "n": int(raw.n_nodes), "nnz": int(len(raw.indices)), "build_s": t_build,
                   "phase_ms": raw.phase_ms, "host_ms": raw.host_ms}, fh)


def _worker(rank, world, port, path, outdir):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gfa2network_amd.shard import HipEngine, build_sharded, file_line_ranges, gather_csr

        eng = HipEngine(0)
        dist.barrier()
        t0 = time.perf_counter()
        lo, hi = file_line_ranges(path, world)[rank]
        buf = eng.read_range(path, lo, hi - lo)
        t_read = time.perf_counter() - t0
        res = build_sharded(buf, engine=eng, gather_names=True, names_root=0, trim=True, **MODE)
        del buf
        t_build = time.perf_counter() - t0 - t_read
        assert res.status == 0, res.status
        dist.barrier()
        t1 = time.perf_counter()
        got = gather_csr(res, None, root=0)
        t_gather = time.perf_counter() - t1
        rec = {"rank": rank, "range_bytes": hi - lo, "rows": [res.row_lo, res.row_hi],
               "slice_nnz": int(res.indices.numel()), "fast_path": res.fast_path, "parse_path": res.parse_path,
               "read_s": t_read, "build_s": t_build, "gather_s": t_gather,
               "a2a_bytes_sent": int(res.a2a_bytes_sent),
               "stages_ms": {k: round(float(v), 3) for k, v in res.timings_ms.items()}}
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
            json.dump(rec, fh)
        if rank == 0:
            indptr, indices, data = got
            d = _digest(indptr, indices, data, res.names_blob, res.names_offsets)
            with open(os.path.join(outdir, "sharded.json"), "w") as fh:
                json.dump({"digest": d, "n": int(res.n_nodes), "nnz": int(len(indices))}, fh)
        else:
            assert got is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("names", ["decimal", "hashed"])
def test_c5_eight_rank_shard_equals_one_gpu(gpu, tmp_path, names):
    import torch.multiprocessing as mp

    from gfa2network_amd import synth

    path = tmp_path / "c5.gfa"
    t0 = time.perf_counter()
    size = synth.write_file(path, N_S, N_L, seed=SEED, names=names, threads=16)
    t_gen = time.perf_counter() - t0
    try:
        mp.spawn(_one_gpu, args=(str(path), str(tmp_path)), nprocs=1, join=True)
        one = json.loads((tmp_path / "one_gpu.json").read_text())
        t1 = time.perf_counter()
        mp.spawn(_worker, args=(WORLD, _free_port(), str(path), str(tmp_path)), nprocs=WORLD, join=True)
        t_shard = time.perf_counter() - t1
        got = json.loads((tmp_path / "sharded.json").read_text())
        ranks = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(WORLD)]
    finally:
        path.unlink()
    rec = {"config": "C5", "names": names, "n_segments": N_S, "n_links": N_L, "file_bytes": size, "world": WORLD,
           "backend": "gloo (8 processes on one MI355X)", "mode": MODE, "generate_s": t_gen,
           "one_gpu": one, "sharded_wall_s": t_shard, "sharded": got, "ranks": ranks}
    out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, f"c5_shard_{names}.json"), "w") as fh:
        json.dump(rec, fh, indent=1)
    assert got["n"] == one["n"] == N_S
    assert sum(r["slice_nnz"] for r in ranks) == one["nnz"]
    assert all(r["fast_path"] == (names == "decimal") for r in ranks)
    for k in ("indptr", "indices", "data", "names_blob", "names_offsets"):
        assert got["digest"][k] == one["digest"][k], f"{k} differs from the single-GPU build"
