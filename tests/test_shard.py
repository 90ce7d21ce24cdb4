"""Sharded build of one file over world_size 2 / 3 gloo ranks on the CPU.

The product's protocol (gfa2network_amd/shard.py: names to owners, owner dedup, global ids,
triplet routing, per-rank CSR slices, stream-order error / warning resolution) driven by the
oracle-backed CPU engine (tests/shard_cpu_engine.py); the gathered result must equal the
oracle's single-file build: node names in id order, and the CSR parse_gfa / convert_format
returns (MAX-SYM or SUM).
"""
import os
import random
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.timeout(600)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gfa(seed, n_s, n_l, shuffle, extra=()):
    r = random.Random(seed)
    names = [f"s{k}" if k % 4 else f"node_{k:06d}_" + "q" * r.randint(0, 20) for k in range(n_s)]
    lines = [f"S\t{n}\t*\n" for n in names]
    for _ in range(n_l):
        a, b = r.choice(names), r.choice(names + ["ghost1", "ghost2"])
        lines.append(f"L\t{a}\t{r.choice('+-')}\t{b}\t{r.choice('+-')}\t*\tRC:i:{r.randint(0, 7)}\n")
    if shuffle:
        r.shuffle(lines)
        lines += [lines[3]] if lines[3].startswith("S") else []
    lines[len(lines) // 2:len(lines) // 2] = list(extra)
    return "".join(lines).encode()


CASES = {
    "s_first": (_gfa(1, 300, 1500, False), {}),
    "shuffled": (_gfa(2, 300, 1500, True), {}),
    "undirected": (_gfa(3, 200, 1000, True), {"directed": False}),
    "bidirected": (_gfa(4, 200, 1000, True), {"bidirected": True}),
    "keep": (_gfa(5, 200, 1000, True), {"bidirected": True, "keep_directed_bidir": True}),
    "asym_weighted_int32": (_gfa(6, 200, 1000, True), {"asymmetric": True, "weight_tag": "RC", "dtype": "int32"}),
    "weighted_int8": (_gfa(7, 150, 900, True), {"weight_tag": "RC", "dtype": "int8"}),
    "bool": (_gfa(8, 150, 900, True), {"dtype": "bool"}),
    "warning": (_gfa(9, 200, 1000, False, extra=["W\tsample\t1\tchr1\t0\t10\t>s1\n"]), {}),
    "error": (_gfa(10, 200, 1000, False, extra=["L\tbad\t+\n"]), {}),
    "tiny": (b"S\ta\t*\nL\ta\t+\tb\t-\t*\n", {}),
}


def _decimal_gfa(seed, n_s, n_l, breaks=None):
    """S lines "1".."N" first, then L lines naming them: the decimal-id fast path; `breaks` spoils
    its premise somewhere (the general protocol must then give the same answer)."""
    r = random.Random(seed)
    lines = [f"S\t{k}\t{'ACGT' * r.randint(0, 3)}\n" for k in range(1, n_s + 1)]
    lines += [f"L\t{r.randint(1, n_s)}\t{r.choice('+-')}\t{r.randint(1, n_s)}\t{r.choice('+-')}\t0M\n"
              for _ in range(n_l)]
    if breaks == "late_s":  # an S line after the edges (in the last range)
        lines.append(f"S\t{n_s + 1}\t*\n")
    if breaks == "ghost":  # an edge key that is no segment
        lines.insert(n_s + n_l // 2, f"L\t{n_s + 5}\t+\t1\t+\t*\n")
    return "".join(lines).encode()


CASES.update({
    "decimal": (_decimal_gfa(11, 400, 2000), {}),
    "decimal_undirected": (_decimal_gfa(12, 400, 2000), {"directed": False}),
    "decimal_bidir": (_decimal_gfa(13, 300, 1500), {"bidirected": True}),
    "decimal_late_s": (_decimal_gfa(14, 300, 1500, "late_s"), {}),
    "decimal_ghost": (_decimal_gfa(15, 300, 1500, "ghost"), {"directed": False}),
})


def _worker(rank, world, port, name, outdir):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch

        from gfa2network_amd.shard import build_sharded, gather_csr, line_ranges
        from oracle import oracle as orc
        from shard_cpu_engine import CpuEngine

        data, mode = CASES[name]
        lo, hi = line_ranges(data, world)[rank]
        buf = torch.from_numpy(np.frombuffer(data[lo:hi], dtype=np.uint8).copy())
        res = build_sharded(buf, engine=CpuEngine(orc), gather_names=True, **mode)
        full = orc.run(data, **mode)
        if full.status:
            assert res.status == full.status, (res.status, full.status)
            if full.status not in (10, 11, 12):
                assert res.err_line == full.err_line, (res.err_line, full.err_line)
            np.save(os.path.join(outdir, f"ok{rank}.npy"), np.zeros(1))
            return
        assert res.status == 0, res.status
        # the decimal-id fast path runs exactly when its premise holds over the whole file
        assert res.fast_path == (name in ("decimal", "decimal_undirected", "decimal_bidir")), (name, res.fast_path)
        assert res.has_warning == full.has_warning and (not full.has_warning or res.warn_line == full.warn_line)
        indptr, indices, vals = gather_csr(res)
        want_names = [bytes(full.names_blob[full.names_offsets[i]:full.names_offsets[i + 1]])
                      for i in range(full.n_nodes)]
        assert res.n_nodes == full.n_nodes and res.names == want_names
        if full.maxsym:
            wp, wi, wd = full.ms_indptr, full.ms_indices, full.ms_data
        else:
            wp, wi, wd = full.sum_indptr, full.sum_indices, full.sum_data
        assert np.array_equal(indptr, wp) and np.array_equal(indices, wi), name
        assert np.asarray(vals).view(np.uint8).tobytes() == np.ascontiguousarray(wd).view(np.uint8).tobytes(), name
        np.save(os.path.join(outdir, f"ok{rank}.npy"), np.zeros(1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", list(CASES))
def test_sharded_build_equals_single_file(oracle_lib, tmp_path, world, name):
    import torch.multiprocessing as mp

    mp.spawn(_worker, args=(world, _free_port(), name, str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"ok{r}.npy").exists()


def test_line_ranges_are_line_aligned_and_cover():
    from gfa2network_amd.shard import line_ranges

    data = _gfa(3, 50, 200, True)
    for g in (1, 2, 3, 5, 8):
        rs = line_ranges(data, g)
        assert rs[0][0] == 0 and rs[-1][1] == len(data)
        for (a, b), (c, _) in zip(rs, rs[1:]):
            assert b == c and (a == b or data[b - 1:b] == b"\n")


def _file_worker(rank, world, port, path, mode, outdir):
    """parse_gfa_sharded through its file entry point: each rank preads only its byte range."""
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import warnings

        from gfa2network_amd.api import finalize, parse_gfa_sharded
        from oracle import oracle as orc
        from shard_cpu_engine import CpuEngine

        data = open(path, "rb").read()
        full = orc.run(data, **mode)
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            A, nodes = parse_gfa_sharded(path, engine=CpuEngine(orc), return_node_list=True, **mode)
        B, bnodes = finalize(orc.to_raw(full, "parse"), dtype=np.dtype(mode.get("dtype", "float64")),
                             return_node_list=True, raw_bytes_id=False, verbose=False)
        assert A.format == B.format and A.shape == B.shape and nodes == bnodes
        if A.format == "coo":
            assert np.array_equal(A.row, B.row) and np.array_equal(A.col, B.col)
        else:
            assert np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
        assert A.data.tobytes() == B.data.tobytes()
        C = parse_gfa_sharded(path, engine=CpuEngine(orc), output="csr", **mode)
        R = orc.to_raw(full, "csr")
        assert np.array_equal(C.indptr, R.indptr) and np.array_equal(C.indices, R.indices)
        np.save(os.path.join(outdir, f"ok{rank}.npy"), np.zeros(1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", ["decimal", "decimal_undirected", "shuffled", "undirected", "warning"])
def test_parse_gfa_sharded_from_file(oracle_lib, tmp_path, world, name):
    """The collective entry point (per-rank pread of its line-aligned byte range, the exchange,
    the gathered result in parse_gfa's format) equals the single-file answer."""
    import torch.multiprocessing as mp

    data, mode = CASES[name]
    path = tmp_path / "in.gfa"
    path.write_bytes(data)
    mp.spawn(_file_worker, args=(world, _free_port(), str(path), mode, str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"ok{r}.npy").exists()


def test_file_line_ranges_match_in_memory_ranges(tmp_path):
    from gfa2network_amd.shard import file_line_ranges, line_ranges

    for seed in range(4):
        data = _gfa(seed, 80, 300, True) + b"S\tlong\t" + b"A" * 70000 + b"\nL\ta\t+\tb\t+\t*"
        path = tmp_path / f"f{seed}.gfa"
        path.write_bytes(data)
        for g in (1, 2, 3, 7, 8):
            assert file_line_ranges(str(path), g, window=4096) == line_ranges(data, g)


def test_scipy_index_dtype_past_int32():
    """The gathered result's index dtype is scipy's (get_index_dtype with check_contents): int32 up
    to 2^31 - 1 entries / nodes, int64 beyond (builders.py:281-283, utils.py:55)."""
    from gfa2network_amd.shard import scipy_index_dtype

    assert scipy_index_dtype(2**31 - 1, 10) == np.int32
    assert scipy_index_dtype(2**31, 10) == np.int64
    assert scipy_index_dtype(0, 2**31) == np.int64
    assert scipy_index_dtype(5, 2**31 - 1) == np.int32


def test_concat_indptr_past_int32():
    """Slice indptrs (each from 0) whose entries total more than 2^31: the global indptr is int64
    and exact — no int32 wrap (three slices of 1.0e9 / 0.9e9 / 0.4e9 entries)."""
    from gfa2network_amd.shard import concat_indptr, scipy_index_dtype

    parts = [np.array([0, 10**9 - 5, 10**9], dtype=np.int32), np.array([0, 9 * 10**8], dtype=np.int32),
             np.array([0], dtype=np.int32), np.array([0, 1, 4 * 10**8], dtype=np.int32)]
    total = 10**9 + 9 * 10**8 + 4 * 10**8
    dt = scipy_index_dtype(total, 5)
    assert dt == np.int64
    ip = concat_indptr(parts, dt)
    assert ip.dtype == np.int64
    assert ip.tolist() == [0, 10**9 - 5, 10**9, 19 * 10**8, 19 * 10**8 + 1, total]
    small = concat_indptr([np.array([0, 2, 3], dtype=np.int32), np.array([0, 4], dtype=np.int32)], np.int32)
    assert small.dtype == np.int32 and small.tolist() == [0, 2, 3, 7]


def _root_worker(rank, world, port, path, mode, root, outdir):
    """parse_gfa_sharded(..., root=k): the result on rank k only, equal to the single-file one."""
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gfa2network_amd.api import finalize, parse_gfa_sharded
        from oracle import oracle as orc
        from shard_cpu_engine import CpuEngine

        data = open(path, "rb").read()
        full = orc.run(data, **mode)
        if full.status:  # a failed build raises on EVERY rank (None would read as success)
            import warnings

            try:
                with warnings.catch_warnings():
                    warnings.simplefilter("ignore")
                    finalize(orc.to_raw(full, "parse"), dtype=np.dtype(mode.get("dtype", "float64")),
                             return_node_list=False, raw_bytes_id=False, verbose=False)
            except Exception as e:  # noqa: BLE001 - the reference's exception, whatever it is
                want = (type(e), str(e))
            for output in ("parse", "csr"):
                try:
                    with warnings.catch_warnings():
                        warnings.simplefilter("ignore")
                        parse_gfa_sharded(path, engine=CpuEngine(orc), output=output, root=root, **mode)
                except Exception as e:  # noqa: BLE001
                    assert (type(e), str(e)) == want, (rank, e, want)
                else:
                    raise AssertionError(f"rank {rank}: no exception")
            np.save(os.path.join(outdir, f"ok{rank}.npy"), np.zeros(1))
            return
        for output in ("parse", "csr"):
            got = parse_gfa_sharded(path, engine=CpuEngine(orc), return_node_list=output == "parse", output=output,
                                    root=root, **mode)
            if rank != root:
                assert got is None
                continue
            if output == "parse":
                A, nodes = got
                B, bnodes = finalize(orc.to_raw(full, "parse"), dtype=np.dtype(mode.get("dtype", "float64")),
                                     return_node_list=True, raw_bytes_id=False, verbose=False)
                assert nodes == bnodes
            else:
                A, B = got, orc.to_raw(full, "csr")
            if A.format == "coo":
                assert np.array_equal(A.row, B.row) and np.array_equal(A.col, B.col)
            else:
                assert np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
                assert A.indptr.dtype == np.int32
            assert np.asarray(A.data).tobytes() == np.asarray(B.data).tobytes()
        np.save(os.path.join(outdir, f"ok{rank}.npy"), np.zeros(1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,root", [("shuffled", 1), ("decimal", 2), ("undirected", 0), ("error", 1)])
def test_parse_gfa_sharded_to_root_only(oracle_lib, tmp_path, name, root):
    import torch.multiprocessing as mp

    data, mode = CASES[name]
    path = tmp_path / "in.gfa"
    path.write_bytes(data)
    mp.spawn(_root_worker, args=(3, _free_port(), str(path), mode, root, str(tmp_path)), nprocs=3, join=True)
    for r in range(3):
        assert (tmp_path / f"ok{r}.npy").exists()


def _want_worker(rank, world, port, paths, outdir):
    """shard="auto" is decided collectively: rank 0's GPU has room, rank 1's does not -> both shard;
    ranks naming different files -> ValueError on every rank (no rank enters the build alone)."""
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gfa2network_amd import api

        size = os.path.getsize(paths[0])
        free = size * api.WORKING_SET_PER_INPUT_BYTE * (4 if rank == 0 else 0.5)
        api._free_hbm = lambda device=None, need=0: int(free)
        assert api._want_shard(paths[0], "auto", 0) is True
        assert api._want_shard(paths[0], "never", 0) is False
        api._free_hbm = lambda device=None, need=0: 10**15
        assert api._want_shard(paths[0], "auto", 0) is False  # fits everywhere
        with pytest.raises(ValueError, match="same file"):
            api._want_shard(paths[rank], "always", 0)
        np.save(os.path.join(outdir, f"ok{rank}.npy"), np.zeros(1))
    finally:
        dist.destroy_process_group()


def test_shard_auto_is_decided_collectively(tmp_path):
    import torch.multiprocessing as mp

    paths = []
    for k in range(2):
        p = tmp_path / f"in{k}.gfa"
        p.write_bytes(CASES["tiny"][0] * (k + 1))
        paths.append(str(p))
    mp.spawn(_want_worker, args=(2, _free_port(), paths, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        assert (tmp_path / f"ok{r}.npy").exists()


@pytest.mark.parametrize("bidirected", [False, True])
def test_decimal_and_gathered_names(bidirected):
    """The node-list helpers of the sharded build: decimal ids by arithmetic (builders.py:190-198
    keys "k" / "k:+", "k:-") and names put in global id order (g2n_gather_names)."""
    from gfa2network_amd import _native as nat

    for n in (0, 2, 8, 10, 18, 20, 198, 200, 2002, 20000):
        blob, offs = nat.decimal_names(n, bidirected)
        want = ([f"{k // 2 + 1}:{'+-'[k & 1]}" for k in range(n)] if bidirected else [str(k + 1) for k in range(n)])
        assert [bytes(blob[offs[i]:offs[i + 1]]).decode() for i in range(n)] == want
    rng = np.random.default_rng(5)
    keys = [bytes(rng.integers(33, 127, rng.integers(0, 40)).astype(np.uint8)) for _ in range(3000)]
    offs = np.zeros(len(keys) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(k) for k in keys])
    blob = np.frombuffer(b"".join(keys), dtype=np.uint8)
    order = rng.permutation(len(keys))
    ob, oo = nat.gather_names(blob, offs, order)
    assert [bytes(ob[oo[i]:oo[i + 1]]) for i in range(len(keys))] == [keys[k] for k in order]


def _range_worker(rank, world, port, outdir):
    """The one-pass decimal protocol on the CPU engine over the range-premise inputs of
    tests/test_gpu_shard.py (S sections spanning ranges, breaks only the range offset or the file's
    S count reveal): every rank takes the same branch, the result is the single-file one."""
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch

        from gfa2network_amd.shard import build_sharded, gather_csr, line_ranges
        from oracle import oracle as orc
        from shard_cpu_engine import CpuEngine
        from test_gpu_shard import _range_cases

        for name, (data, fast) in _range_cases(world).items():
            lo, hi = line_ranges(data, world)[rank]
            buf = torch.from_numpy(np.frombuffer(data[lo:hi], dtype=np.uint8).copy())
            res = build_sharded(buf, engine=CpuEngine(orc), gather_names=True, names_root=0)
            assert res.status == 0 and res.fast_path == fast, (name, rank)
            indptr, indices, vals = gather_csr(res)
            if rank == 0:
                full = orc.run(data)
                assert np.array_equal(indptr, full.ms_indptr) and np.array_equal(indices, full.ms_indices), name
                assert res.n_nodes == full.n_nodes, name
        np.save(os.path.join(outdir, f"ok{rank}.npy"), np.zeros(1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_range_premise_one_pass(oracle_lib, tmp_path, world):
    import torch.multiprocessing as mp

    mp.spawn(_range_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"ok{r}.npy").exists()


def _gz_files(data: bytes, tmp_path):
    """The same text as several gzip layouts: many members (more than ranks), BGZF, fewer members than
    ranks (some ranks inflate nothing), one member (rank 0 inflates it all; the all-to-all spreads it),
    zero padding after the last member."""
    import gzip
    import struct
    import zlib

    out = {}

    def members(k):
        step = max(1, -(-len(data) // k))
        return b"".join(gzip.compress(data[i:i + step]) for i in range(0, len(data), step))
    out["many"] = members(11)
    out["two"] = members(2)
    out["one"] = gzip.compress(data)
    body = bytearray()
    for k in range(0, len(data), 4000):
        chunk = data[k:k + 4000]
        co = zlib.compressobj(6, zlib.DEFLATED, -zlib.MAX_WBITS)
        z = co.compress(chunk) + co.flush()
        body += (b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", 25 + len(z))
                 + z + struct.pack("<II", zlib.crc32(chunk), len(chunk)))
    out["bgzf"] = bytes(body) + bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    out["padded"] = members(5) + b"\x00" * 64
    paths = {}
    for name, blob in out.items():
        p = tmp_path / f"{name}.gfa.gz"
        p.write_bytes(blob)
        paths[name] = str(p)
    return paths


def _gz_rank_worker(rank, world, port, paths, data_path, outdir):
    """gz_rank_text: each rank inflates only the members starting in its share of the compressed bytes
    and ends with exactly line_ranges' range of the whole inflated text; parse_gfa_sharded over it
    equals the oracle's one-piece build."""
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gfa2network_amd import shard
        from gfa2network_amd.api import finalize, parse_gfa_sharded
        from oracle import oracle as orc
        from shard_cpu_engine import CpuEngine

        data = open(data_path, "rb").read()
        want = shard.line_ranges(data, world)[rank]
        full = orc.run(data)
        B, bnodes = finalize(orc.to_raw(full, "parse"), dtype=np.dtype("float64"), return_node_list=True,
                             raw_bytes_id=False, verbose=False)
        for name, path in paths.items():
            got = shard.gz_rank_text(path, CpuEngine(orc))  # ("one": rank 0 inflates it, the others nothing)
            assert got is not None, name
            buf, n = got
            assert n == len(data) and bytes(buf.numpy()) == data[want[0]:want[1]], (name, rank)
            A, nodes = parse_gfa_sharded(path, engine=CpuEngine(orc), return_node_list=True)
            assert nodes == bnodes and np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
        np.save(os.path.join(outdir, f"ok{rank}.npy"), np.zeros(1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 5])
def test_sharded_gzip_inflates_per_rank(oracle_lib, tmp_path, world):
    import torch.multiprocessing as mp

    data = _gfa(41, 300, 2500, True)
    data_path = tmp_path / "in.gfa"
    data_path.write_bytes(data)
    paths = _gz_files(data, tmp_path)
    mp.spawn(_gz_rank_worker, args=(world, _free_port(), paths, str(data_path), str(tmp_path)), nprocs=world,
             join=True)
    for r in range(world):
        assert (tmp_path / f"ok{r}.npy").exists()


def test_gz_member_candidates(tmp_path):
    """gz_member_at_or_after finds the next real member start (not a 1f 8b 08 inside a name or in
    deflate data that zlib refuses), or the file size."""
    import gzip

    from gfa2network_amd.shard import gz_member_at_or_after

    a = gzip.compress(b"S\t\x1f\x8b\x08fake\t*\n" * 50)
    b = gzip.compress(b"L\tx\t+\ty\t+\t*\n" * 50)
    p = tmp_path / "x.gz"
    p.write_bytes(a + b)
    size = len(a) + len(b)
    assert gz_member_at_or_after(str(p), 0, size) == 0
    assert gz_member_at_or_after(str(p), 1, size) == len(a)
    assert gz_member_at_or_after(str(p), len(a), size) == len(a)
    assert gz_member_at_or_after(str(p), len(a) + 1, size) == size
