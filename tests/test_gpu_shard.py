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
        cases = [(name, data, mode, False) for name, (data, modes) in _inputs().items() for mode in modes]
        if world == 1:  # the one-rank slot partition declining (an overfull bucket): the stream-order route
            cases += [(name, data, mode, True) for name, data, mode, _ in cases if name == "synthetic"]
        for name, data, mode, decline in cases:
            lo, hi = line_ranges(data, world)[rank]
            buf = torch.from_numpy(np.frombuffer(data[lo:hi], dtype=np.uint8).copy()).to(eng.device)
            if decline:
                eng.csr_slots = lambda *a, **k: None
            res = build_sharded(buf, engine=eng, gather_names=True, **mode)
            if decline:
                del eng.csr_slots
                assert res.coo_layout == "stream", (name, mode)
            assert res.status == 0, (name, mode, res.status)
            assert res.fast_path == (name == "synthetic"), (name, mode)  # decimal ids: no id exchange
            if res.fast_path and not mode.get("bidirected") and not decline:  # the range parse's group slots,
                assert res.coo_layout == "group_slots", (name, mode)  # routed / assembled in place
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


@pytest.mark.parametrize("world", [1, 2, 3])
def test_gpu_sharded_build_equals_single_file(gpu, oracle_lib, tmp_path, world):
    import torch.multiprocessing as mp

    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"ok{r}.npy").exists()


def _file_worker(rank, world, port, path, backend, outdir):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch

    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gfa2network_amd import convert_format, parse_gfa, parse_gfa_sharded

        for mode in ({}, {"directed": False}, {"bidirected": True, "weight_tag": "RC"}):
            A, nodes = parse_gfa_sharded(path, return_node_list=True, **mode)
            B, bnodes = parse_gfa(path, build_graph=False, build_matrix=True, return_node_list=True, shard="never",
                                  **mode)
            assert A.format == B.format and nodes == bnodes, mode
            if A.format == "coo":
                assert np.array_equal(A.row, B.row) and np.array_equal(A.col, B.col), mode
            else:
                assert np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices), mode
            assert A.data.tobytes() == B.data.tobytes(), mode
            C = parse_gfa_sharded(path, output="csr", **mode)
            D = convert_format(B, "csr")
            assert np.array_equal(C.indptr, D.indptr) and C.data.tobytes() == D.data.tobytes(), mode
            # parse_gfa's own dispatch: shard="always" takes the same collective path
            E = parse_gfa(path, build_graph=False, build_matrix=True, shard="always", **mode)
            assert E.format == B.format and E.data.tobytes() == B.data.tobytes(), mode
        np.save(os.path.join(outdir, f"ok{rank}.npy"), np.zeros(1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,backend", [(2, "gloo"), (3, "gloo"), (1, "nccl")])
def test_gpu_parse_gfa_sharded_from_file(gpu, tmp_path, world, backend):
    """The collective entry point on the HIP engine: each rank preads its byte range of the file
    straight into HBM (g2n_upload_file_range); the result equals the single-GPU parse_gfa.  The
    nccl (RCCL) case runs the exchange on device tensors (one rank: the box has one GPU, and RCCL
    refuses two ranks on one device)."""
    import torch.multiprocessing as mp

    from gfa2network_amd import synth

    path = tmp_path / "in.gfa"
    path.write_bytes(synth.host_bytes(60_000, 240_000, seed=9, rc_tag=True))
    mp.spawn(_file_worker, args=(world, _free_port(), str(path), backend, str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"ok{r}.npy").exists()


@pytest.mark.parametrize("n_ranks", [1, 2, 3, 8, 100, 256, 300])
def test_gpu_route_triplets_stable_partition(gpu, n_ranks):
    """g2n_route_triplets (the owner partition of g2n_route.hip; > 256 ranks the sort path) equals
    numpy's stable partition by owner = floor(row * R / n_global): stream order kept per owner, with
    and without an id map, transposed, values of 1, 4 and 8 bytes or none."""
    import torch

    from gfa2network_amd.shard import HipEngine

    rng = np.random.default_rng(n_ranks)
    n, n_global = 300_000 + n_ranks, 1_000_003
    rows = rng.integers(0, n_global, n).astype(np.int32)
    cols = rng.integers(0, n_global, n).astype(np.int32)
    perm = rng.permutation(n_global).astype(np.uint32)
    eng = HipEngine(0)
    try:
        for use_map in (False, True):
            for transposed in (False, True):
                for dt in ("float64", "int32", "int8", None):
                    data = None if dt is None else rng.integers(-100, 100, n).astype(dt)
                    r, c = (perm[rows].astype(np.int64), perm[cols].astype(np.int64)) if use_map else (rows, cols)
                    if transposed:
                        r, c = c, r
                    owner = np.asarray(r, dtype=np.int64) * n_ranks // n_global
                    order = np.argsort(owner, kind="stable")
                    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(eng.device)  # noqa: E731
                    rr, cc, dd, st = eng.route_triplets(d(rows), d(cols), None if data is None else d(data),
                                                        dt or "float64", d(perm.view(np.int32)) if use_map else None,
                                                        n_global, n_ranks, transposed)
                    key = (use_map, transposed, dt)
                    assert np.array_equal(rr.cpu().numpy(), np.asarray(r)[order]), key
                    assert np.array_equal(cc.cpu().numpy(), np.asarray(c)[order]), key
                    if data is not None:
                        assert np.array_equal(dd.cpu().numpy(), data[order]), key
                    else:
                        assert dd is None
                    want = np.searchsorted(owner[order], np.arange(n_ranks + 1))
                    assert np.array_equal(st.cpu().numpy(), want), key
        # empty input
        e = torch.zeros(0, dtype=torch.int32, device=eng.device)
        rr, cc, dd, st = eng.route_triplets(e, e, None, "float64", None, n_global, n_ranks, False)
        assert rr.numel() == 0 and np.array_equal(st.cpu().numpy(), np.zeros(n_ranks + 1))
    finally:
        eng.close()


def _gz_worker(rank, world, port, paths, outdir):
    """parse_gfa_sharded on .gz files: a clean one equals the single-GPU build; a truncated / corrupt
    one raises exactly what the single-GPU parse_gfa raises (gzip.py's exception and message, after
    the lines before the failure were parsed) on every rank."""
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import warnings

        from gfa2network_amd import parse_gfa, parse_gfa_sharded

        for path in paths:
            outs = []
            for fn in (lambda: parse_gfa_sharded(path, return_node_list=True),
                       lambda: parse_gfa(path, build_graph=False, build_matrix=True, return_node_list=True)):
                with warnings.catch_warnings(record=True) as w:
                    warnings.simplefilter("always")
                    try:
                        outs.append(("ok", fn(), [str(x.message) for x in w]))
                    except Exception as exc:  # noqa: BLE001 - compared below
                        outs.append(("exc", (type(exc), str(exc)), [str(x.message) for x in w]))
            (ka, va, wa), (kb, vb, wb) = outs
            assert ka == kb and wa == wb, (path, outs)
            if ka == "exc":
                assert va == vb, (path, va, vb)
            else:
                (A, na), (B, nb) = va, vb
                assert na == nb and np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
                assert A.data.tobytes() == B.data.tobytes()
        np.save(os.path.join(outdir, f"ok{rank}.npy"), np.zeros(1))
    finally:
        dist.destroy_process_group()


def test_gpu_sharded_gzip_clean_and_corrupt(gpu, tmp_path):
    import gzip
    import zlib

    import torch.multiprocessing as mp

    from gfa2network_amd import synth

    data = synth.host_bytes(20_000, 80_000, seed=23)
    good = gzip.compress(data[:len(data) // 2]) + gzip.compress(data[len(data) // 2:])
    paths = []
    for name, blob in (("good.gfa.gz", good), ("trunc.gfa.gz", good[:len(good) * 3 // 4]),
                       ("crc.gfa.gz", good[:-8] + (zlib.crc32(b"x") & 0xFFFFFFFF).to_bytes(4, "little") + good[-4:]),
                       ("garbage.gfa.gz", good[:100] + bytes(range(256)) * 8 + good[2148:])):
        p = tmp_path / name
        p.write_bytes(blob)
        paths.append(str(p))
    mp.spawn(_gz_worker, args=(2, _free_port(), paths, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        assert (tmp_path / f"ok{r}.npy").exists()


def _range_cases(world):
    """Decimal-id inputs whose S section spans more than one byte range (S lines before a range,
    S lines inside a later range), each range many 32 KiB tiles, and premise breaks that only the
    range offset (s_base) or the whole file's S count (N) can see: the sharded tile-local lean parse
    (k_tile_lean + k_tile_lean_check with s_base / n_seg_all) must take exactly the canonical ones."""
    from gfa2network_amd.shard import line_ranges

    r = random.Random(21)
    n_s, n_l = 60_000, 100_000
    S = [f"S\t{k}\t{'ACGT' * r.randint(5, 15)}\n" for k in range(1, n_s + 1)]
    L = [f"L\t{r.randint(1, n_s)}\t{r.choice('+-')}\t{r.randint(1, n_s)}\t{r.choice('+-')}\t0M\n" for _ in range(n_l)]
    base = "".join(S + L).encode()
    lo1, hi1 = line_ranges(base, world)[1]
    # S lines whose bytes start inside range 1
    pos, in_r1 = 0, []
    for i, x in enumerate(S):
        if lo1 <= pos < hi1:
            in_r1.append(i)
        pos += len(x)
    assert in_r1 and in_r1[0] > 0, "range 1 must start inside the S section"
    shifted = list(S)
    for i in in_r1:  # range 1's S names all one too high: consistent inside the range, wrong for its s_base
        shifted[i] = f"S\t{i + 2}\t{S[i].split(chr(9))[2]}"
    assert sum(map(len, shifted)) == sum(map(len, S))
    renamed = list(S)
    renamed[in_r1[len(in_r1) // 2]] = f"S\t{in_r1[len(in_r1) // 2] + 1}x\t*\n"
    half = len(L) // 10
    return {  # name -> (bytes, fast path expected)
        "canonical": (base, True),
        "edge_names_n_last_range": (base + f"L\t{n_s}\t+\t1\t-\t0M\n".encode(), True),
        "s_names_off_by_range_base": ("".join(shifted + L).encode(), False),
        "s_renamed_in_range1": ("".join(renamed + L).encode(), False),
        "edge_beyond_n_last_range": (base + f"L\t{n_s + 1}\t+\t1\t-\t0M\n".encode(), False),
        "s_after_edges": ("".join(S[:n_s // 2] + L[:half] + S[n_s // 2:] + L[half:]).encode(), False),
    }


def _range_worker(rank, world, port, outdir):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch

        from gfa2network_amd.shard import HipEngine, build_sharded, gather_csr, line_ranges
        from oracle import oracle as orc

        eng = HipEngine(0)
        for name, (data, fast) in _range_cases(world).items():
            lo, hi = line_ranges(data, world)[rank]
            assert hi - lo > 8 * 32768, (name, rank, hi - lo)
            buf = torch.from_numpy(np.frombuffer(data[lo:hi], dtype=np.uint8).copy()).to(eng.device)
            for mode in ({}, {"directed": False}, {"dtype": "int8"}):
                res = build_sharded(buf, engine=eng, gather_names=True, names_root=0, **mode)
                assert res.status == 0, (name, mode, res.status)
                assert res.fast_path == fast, (name, mode, rank)
                if fast:  # the one-pass lean parse, not K1 + the tile parse
                    assert res.parse_path == "tile_local", (name, mode, rank, res.parse_path)
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
def test_gpu_sharded_tile_local_range_premise(gpu, oracle_lib, tmp_path, world):
    """Sharded decimal-id ranges take the tile-local lean parse; premise breaks visible only through
    the range's S offset or the file's S count fall back to the general protocol.  Always the oracle's
    single-file answer."""
    import torch.multiprocessing as mp

    mp.spawn(_range_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"ok{r}.npy").exists()


@pytest.mark.parametrize("mode", [{}, {"directed": False}, {"asymmetric": True}, {"dtype": "int8"},
                                  {"bidirected": True, "weight_tag": "RC"}])
def test_gpu_chunked_single_gpu_build(gpu, oracle_lib, tmp_path, mode):
    """parse_gfa(..., chunk_bytes=...) on one GPU: the file pread and parsed range by range
    (shard.build_chunked: into global decimal ids, or — bidirected / weighted builds, hashed names —
    with local ids merged into one dictionary chunk by chunk), the CSR / COO built once — equal to
    the oracle's one-piece build bit for bit, at 3 and at ~40 ranges."""
    from gfa2network_amd import parse_gfa, synth
    from gfa2network_amd.api import finalize

    data = synth.host_bytes(200_000, 800_000, seed=31, rc_tag=bool(mode.get("weight_tag")))
    path = tmp_path / "in.gfa"
    path.write_bytes(data)
    full = oracle_lib.run(data, **mode)
    B, bnodes = finalize(oracle_lib.to_raw(full, "parse"), dtype=np.dtype(mode.get("dtype", "float64")),
                         return_node_list=True, raw_bytes_id=False, verbose=False)
    for chunk in (len(data) // 3 + 1, 600_000):
        A, nodes = parse_gfa(str(path), build_graph=False, build_matrix=True, return_node_list=True,
                             chunk_bytes=chunk, **mode)
        assert A.format == B.format and A.shape == B.shape and nodes == bnodes, chunk
        if A.format == "coo":
            assert np.array_equal(A.row, B.row) and np.array_equal(A.col, B.col)
        else:
            assert np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
        assert A.data.tobytes() == B.data.tobytes()
    hashed = data.replace(b"S\t7\t", b"S\tx7\t", 1).replace(b"\t7\t+\t", b"\tx7\t+\t")
    path.write_bytes(hashed)
    full = oracle_lib.run(hashed, **mode)
    B, bnodes = finalize(oracle_lib.to_raw(full, "parse"), dtype=np.dtype(mode.get("dtype", "float64")),
                         return_node_list=True, raw_bytes_id=False, verbose=False)
    A, nodes = parse_gfa(str(path), build_graph=False, build_matrix=True, return_node_list=True,
                         chunk_bytes=600_000, **mode)
    assert A.format == B.format and A.data.tobytes() == B.data.tobytes() and nodes == bnodes
    if A.format == "csr":
        assert np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
    else:
        assert np.array_equal(A.row, B.row) and np.array_equal(A.col, B.col)


def _gz_variants(data: bytes, tmp_path):
    """The same text as multi-member gzip, BGZF (bench.write_bgzf's layout) and one gzip member."""
    import gzip
    import struct
    import zlib

    out = {}
    p = tmp_path / "multi.gfa.gz"
    step = max(1, len(data) // 5)
    p.write_bytes(b"".join(gzip.compress(data[k:k + step]) for k in range(0, len(data), step)))
    out["multi_member"] = p
    body = bytearray()
    for k in range(0, len(data), 65280):
        chunk = data[k:k + 65280]
        co = zlib.compressobj(6, zlib.DEFLATED, -zlib.MAX_WBITS)
        z = co.compress(chunk) + co.flush()
        body += (b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", 12 + 6 + len(z) + 8 - 1)
                 + z + struct.pack("<II", zlib.crc32(chunk), len(chunk)))
    body += bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    p = tmp_path / "bgzf.gfa.gz"
    p.write_bytes(bytes(body))
    out["bgzf"] = p
    p = tmp_path / "single.gfa.gz"
    p.write_bytes(gzip.compress(data))
    out["single_member"] = p
    return out


@pytest.mark.parametrize("mode", [{}, {"directed": False}, {"bidirected": True, "weight_tag": "RC"}])
def test_gpu_chunked_gzip_and_default_route(gpu, oracle_lib, tmp_path, monkeypatch, mode):
    """The one-GPU chunked build for every input kind on the HIP engine: .gz files
    (multi-member, BGZF, one member) inflated on the host and chunked from host memory with
    chunk_bytes; then the DEFAULT parse_gfa (no chunk_bytes, shard="never") on a plain file and a .gz
    with the GPU's free HBM reported below the input's working set — it chunks by itself (sized from
    the reported free memory) — and a file object; all bit-exact against the oracle's one-piece build."""
    from gfa2network_amd import api, parse_gfa, synth
    from gfa2network_amd.api import finalize

    data = synth.host_bytes(100_000, 400_000, seed=41, rc_tag=bool(mode.get("weight_tag")))
    full = oracle_lib.run(data, **mode)
    B, bnodes = finalize(oracle_lib.to_raw(full, "parse"), dtype=np.dtype("float64"), return_node_list=True,
                         raw_bytes_id=False, verbose=False)

    def check(A, nodes, what):
        assert A.format == B.format and A.shape == B.shape and nodes == bnodes, what
        if A.format == "coo":
            assert np.array_equal(A.row, B.row) and np.array_equal(A.col, B.col), what
        else:
            assert np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices), what
        assert A.data.tobytes() == B.data.tobytes(), what

    gz = _gz_variants(data, tmp_path)
    for kind, p in gz.items():
        A, nodes = parse_gfa(str(p), build_graph=False, build_matrix=True, return_node_list=True,
                             chunk_bytes=len(data) // 4 + 1, **mode)
        check(A, nodes, kind)
    plain = tmp_path / "in.gfa"
    plain.write_bytes(data)
    calls = []
    real = api._parse_gfa_chunked
    monkeypatch.setattr(api, "_parse_gfa_chunked", lambda *a, **k: calls.append(a[1]) or real(*a, **k))
    monkeypatch.setattr(api, "_free_hbm", lambda device=0, need=0: len(data) * 2)  # the working set does not fit
    monkeypatch.setattr(api, "_chunk_plan", lambda size, device: (len(data) // 3 + 1) if size * 8 > len(data) * 2 else 0)
    import io

    for what, src in (("plain", str(plain)), ("gz", str(gz["multi_member"])), ("fileobj", io.BytesIO(data))):
        n = len(calls)
        A, nodes = parse_gfa(src, build_graph=False, build_matrix=True, return_node_list=True, **mode)
        assert len(calls) == n + 1, f"{what}: the default route did not chunk"
        check(A, nodes, what)


@pytest.mark.parametrize("mode", [{}, {"directed": False, "weight_tag": "RC", "dtype": "float32"}])
def test_gpu_chunked_row_bands_and_errors(gpu, oracle_lib, tmp_path, mode):
    """The chunked build's whole-matrix CSR in row bands on the HIP engine (g2n_route_triplets by band +
    g2n_csr_from_coo_pair per band) equals one piece; and an error / warning in a later chunk comes out
    as one piece raises / emits it."""
    import warnings

    from gfa2network_amd import synth
    from gfa2network_amd.api import _dtype_of, _parse_gfa_chunked, finalize

    data = synth.host_bytes(50_000, 200_000, seed=43, rc_tag=True)
    path = tmp_path / "in.gfa"
    path.write_bytes(data)
    dt = mode.get("dtype", "float64")
    kw = dict(directed=mode.get("directed", True), weight_tag=mode.get("weight_tag"), verbose=False, bidirected=False,
              keep_directed_bidir=False, strip_orientation=False, dt=_dtype_of(dt), asymmetric=False,
              raw_bytes_id=False, return_node_list=True, device=0)
    full = oracle_lib.run(data, **mode)
    B, bnodes = finalize(oracle_lib.to_raw(full, "parse"), dtype=np.dtype(dt), return_node_list=True,
                         raw_bytes_id=False, verbose=False)
    for bands in (3, 7):
        A, nodes = _parse_gfa_chunked(str(path), len(data) // 4 + 1, bands=bands, **kw)
        assert nodes == bnodes and A.format == B.format
        if A.format == "csr":
            assert np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
        else:
            assert np.array_equal(A.row, B.row) and np.array_equal(A.col, B.col)
        assert A.data.tobytes() == B.data.tobytes()
    cut = data.index(b"\nL\t", len(data) * 3 // 4) + 1
    for extra, exc in ((b"W\tsample\t1\tchr1\t0\t10\t>s1\n", None), (b"L\tbroken\n", ValueError)):
        bad = data[:cut] + extra + data[cut:]
        path.write_bytes(bad)
        o = oracle_lib.run(bad, **mode)
        with warnings.catch_warnings(record=True) as w1:
            warnings.simplefilter("always")
            if exc:
                with pytest.raises(exc) as e1:
                    _parse_gfa_chunked(str(path), len(bad) // 5 + 1, **kw)
            else:
                A, nodes = _parse_gfa_chunked(str(path), len(bad) // 5 + 1, **kw)
        with warnings.catch_warnings(record=True) as w2:
            warnings.simplefilter("always")
            if exc:
                with pytest.raises(exc) as e2:
                    finalize(oracle_lib.to_raw(o, "parse"), dtype=np.dtype(dt), return_node_list=True,
                             raw_bytes_id=False, verbose=False)
                assert str(e1.value) == str(e2.value)
            else:
                B2, n2 = finalize(oracle_lib.to_raw(o, "parse"), dtype=np.dtype(dt), return_node_list=True,
                                  raw_bytes_id=False, verbose=False)
                assert nodes == n2 and A.data.tobytes() == B2.data.tobytes()
        assert [str(x.message) for x in w1] == [str(x.message) for x in w2]


# the cross-chunk error ordering on the HIP engine (the CPU engine covers it in
# tests/test_chunked.py): a cast error kept while later chunks parse and a later parse error winning;
# the warning resolved across chunks, then a 0x80-led unsupported record in a later chunk (the
# reference decodes it for its warning only if no warning came first: parser.py:125-131)
GPU_CHUNK_ERRORS = {
    "cast_then_parse_error": (["L\ts1\t+\ts2\t+\t*\tRC:i:300\n"] + ["L\ts3\t+\ts1\t+\t*\n"] * 300 + ["L\tq\n"],
                              {"weight_tag": "RC", "dtype": "int8"}),
    "cast_int8": (["L\ts1\t+\ts2\t+\t*\tRC:i:300\n"], {"weight_tag": "RC", "dtype": "int8"}),
    "warning_then_nonascii": (["W\tsample\t1\tchr1\t0\t10\t>s1\n"] + ["L\ts1\t+\ts2\t+\t*\n"] * 300
                              + ["éx\tnot a record\n"], {}),
    "warning_then_error": (["W\tsample\n"] + ["L\ts1\t+\ts2\t+\t*\n"] * 200 + ["L\tbad\n"], {}),
}


@pytest.mark.parametrize("case", sorted(GPU_CHUNK_ERRORS))
@pytest.mark.parametrize("chunk", [300, 2500])
def test_gpu_chunked_error_order_across_chunks(gpu, oracle_lib, tmp_path, case, chunk):
    """The HIP engine's chunked general build (_chunked_general with the device key set) resolves
    errors, cast errors and the one-shot warning across chunks as the one-piece build does."""
    import sys

    sys.path.insert(0, os.path.dirname(__file__))
    from test_chunked import _named_gfa, _one_piece, _outcome, _same

    from gfa2network_amd.api import _dtype_of, _parse_gfa_chunked

    extra, mode = GPU_CHUNK_ERRORS[case]
    data = _named_gfa(33, 150, 700, True, extra)
    path = tmp_path / "in.gfa"
    path.write_bytes(data)
    kw = dict(directed=mode.get("directed", True), weight_tag=mode.get("weight_tag"), verbose=False, bidirected=False,
              keep_directed_bidir=False, strip_orientation=False, dt=_dtype_of(mode.get("dtype", "float64")),
              asymmetric=False, raw_bytes_id=False, return_node_list=True, device=0)
    _same(_outcome(lambda: _parse_gfa_chunked(str(path), chunk, **kw)), _one_piece(oracle_lib, data, mode))


_NO_TORCH_SCRIPT = r'''
import sys
sys.modules["torch"] = None  # any "import torch" on this path raises ImportError
import json
import numpy as np
from gfa2network_amd import api, parse_gfa

path, out, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
api._free_hbm = lambda device=0, need=0: n * 2  # the working set (8 x the input) does not fit
api._chunk_plan = lambda size, device: (n // 3 + 1) if size * 8 > n * 2 else 0
res = {}
for k, mode in enumerate(json.loads(sys.argv[4])):
    A, nodes = parse_gfa(path, build_graph=False, build_matrix=True, return_node_list=True, **mode)
    arrs = [A.row, A.col] if A.format == "coo" else [A.indptr, A.indices]
    np.savez(f"{out}_{k}.npz", a=arrs[0], b=arrs[1], data=A.data, fmt=A.format,
             names=np.frombuffer("\n".join(nodes).encode(), dtype=np.uint8))
dt = api._dtype_of("float64")
A, nodes = api._parse_gfa_chunked(path, n // 4 + 1, directed=True, weight_tag=None, verbose=False, bidirected=False,
                                  keep_directed_bidir=False, strip_orientation=False, dt=dt, asymmetric=False,
                                  raw_bytes_id=False, return_node_list=True, device=0, bands=3)
np.savez(f"{out}_bands.npz", a=A.indptr, b=A.indices, data=A.data, fmt=A.format,
         names=np.frombuffer("\n".join(nodes).encode(), dtype=np.uint8))
print("torch imported:", "torch" in sys.modules and sys.modules["torch"] is not None)
'''


@pytest.mark.parametrize("names", ["decimal", "hashed"])
def test_gpu_chunked_build_without_torch(gpu, oracle_lib, tmp_path, names):
    """The one-GPU route for an input past its working set (a lowered free-memory report, as in
    test_gpu_chunked_gzip_and_default_route) runs with torch made unimportable:
    HipEngine(torch_buffers=False) keeps its buffers as DevBuf arrays through the HIP runtime —
    decimal chunks, merged-dictionary chunks with the device key set, the whole-matrix CSR, a COO
    result and the row-band assembly — each bit for bit against the oracle's one-piece build."""
    import json
    import subprocess
    import sys

    from gfa2network_amd import synth
    from gfa2network_amd.api import finalize

    data = synth.host_bytes(100_000, 400_000, seed=47, rc_tag=True, names=names)
    path = tmp_path / "in.gfa"
    path.write_bytes(data)
    modes = [{}, {"directed": False}, {"weight_tag": "RC"}, {"bidirected": True, "directed": False}]
    out = str(tmp_path / "r")
    env = dict(os.environ)
    env["PYTHONPATH"] = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", _NO_TORCH_SCRIPT, str(path), out, str(len(data)), json.dumps(modes)],
                       env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "torch imported: False" in p.stdout
    for k, mode in enumerate(modes + [{}]):
        got = np.load(f"{out}_{k if k < len(modes) else 'bands'}.npz")
        o = oracle_lib.run(data, **mode)
        B, bnodes = finalize(oracle_lib.to_raw(o, "parse"), dtype=np.dtype("float64"), return_node_list=True,
                             raw_bytes_id=False, verbose=False)
        assert str(got["fmt"]) == B.format, mode
        if B.format == "coo":
            assert np.array_equal(got["a"], B.row) and np.array_equal(got["b"], B.col), mode
        else:
            assert np.array_equal(got["a"], B.indptr) and np.array_equal(got["b"], B.indices), mode
        assert got["data"].tobytes() == B.data.tobytes(), mode
        assert got["names"].tobytes() == "\n".join(bnodes).encode(), mode
