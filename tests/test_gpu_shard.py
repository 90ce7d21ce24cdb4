"""Sharded build with the HIP engine: 2-3 ranks (processes) on the box's GPU exchanging over
gloo, against the oracle's single-file build — names in id order and the CSR bit for bit,
including weighted float64 sums whose order depends on scipy's global has_sorted_indices."""
import os
import random
import socket

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs():
    from gfa2network_amd import synth

    r = random.Random(4)
    names = [f"n{k}" for k in range(3000)]
    lines = [f"S\t{n}\t*\n" for n in names]
    vals = ["1e16", "1", "-1e16", "0.1", "3.3", "-2.7", "7.25"]
    for _ in range(20000):  # hub rows (> 16 entries) with order-sensitive float sums
        a = r.choice(names[:40])
        lines.append(f"L\t{a}\t+\t{r.choice(names)}\t-\t*\tRC:f:{r.choice(vals)}\n")
    r.shuffle(lines)
    return {
        "synthetic": (synth.host_bytes(100_000, 400_000, seed=3, rc_tag=True), [{}, {"bidirected": True},
                                                                                  {"directed": False}]),
        "shuffled_float_sums": ("".join(lines).encode(), [{"weight_tag": "RC"}, {"weight_tag": "RC",
                                                                                 "directed": False,
                                                                                 "dtype": "float32"}]),
    }


def _worker(rank, world, port, outdir):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch

        from gfa2network_amd.shard import HipEngine, build_sharded, gather_csr, line_ranges
        from oracle import oracle as orc

        eng = HipEngine(0)
        for name, (data, modes) in _inputs().items():
            lo, hi = line_ranges(data, world)[rank]
            buf = torch.from_numpy(np.frombuffer(data[lo:hi], dtype=np.uint8).copy()).to(eng.device)
            for mode in modes:
                res = build_sharded(buf, engine=eng, gather_names=True, **mode)
                assert res.status == 0, (name, mode, res.status)
                indptr, indices, vals = gather_csr(res)
                if rank != 0:
                    continue
                full = orc.run(data, **mode)
                want = [bytes(full.names_blob[full.names_offsets[i]:full.names_offsets[i + 1]])
                        for i in range(full.n_nodes)]
                assert res.names == want, (name, mode)
                wp, wi, wd = ((full.ms_indptr, full.ms_indices, full.ms_data) if full.maxsym
                              else (full.sum_indptr, full.sum_indices, full.sum_data))
                assert np.array_equal(indptr, wp) and np.array_equal(indices, wi), (name, mode)
                assert vals.tobytes() == np.ascontiguousarray(wd).tobytes(), (name, mode)
        eng.close()
        np.save(os.path.join(outdir, f"ok{rank}.npy"), np.zeros(1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gpu_sharded_build_equals_single_file(gpu, oracle_lib, tmp_path, world):
    import torch.multiprocessing as mp

    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"ok{r}.npy").exists()
