"""One file built on one GPU in line-aligned chunks (shard.build_chunked, parse_gfa's chunked mode)
equals the one-piece build — here on the CPU engine (the oracle per range, scipy for the CSR), on
the HIP engine in test_gpu_shard.py.  Chunk sizes from 97 bytes (dozens of ranges, S sections and
edge sections split anywhere) to the whole file, decimal names (one-pass range parse) and any names
(chunks merged into one dictionary); a parse error or warning declines (None) so the caller builds in
one piece."""
import random

import numpy as np
import pytest


def _decimal_gfa(seed, n_s, n_l, breaks=None):
    r = random.Random(seed)
    lines = [f"S\t{k}\t{'ACGT' * r.randint(0, 3)}\n" for k in range(1, n_s + 1)]
    lines += [f"L\t{r.randint(1, n_s)}\t{r.choice('+-')}\t{r.randint(1, n_s)}\t{r.choice('+-')}\t0M\n"
              for _ in range(n_l)]
    if breaks == "late_s":  # an S line after the edges
        lines.append(f"S\t{n_s + 1}\t*\n")
    if breaks == "ghost":  # an edge key that is no segment
        lines.insert(n_s + n_l // 2, f"L\t{n_s + 5}\t+\t1\t+\t*\n")
    if breaks == "offset":  # S names start at 2
        lines = [ln.replace(f"S\t{k}\t", f"S\t{k + 1}\t", 1) if ln.startswith("S") else ln
                 for k, ln in zip(range(1, len(lines) + 1), lines)]
    if breaks == "hashed":
        lines[5] = "S\tx5\t*\n"
    if breaks == "error":
        lines.insert(n_s + 7, "L\t1\t+\n")
    return "".join(lines).encode()


def _chunked(path, chunk, mode):
    from gfa2network_amd.api import _dtype_of, _parse_gfa_chunked
    from oracle import oracle as orc
    from shard_cpu_engine import CpuEngine

    dt = _dtype_of(mode.get("dtype", "float64"))
    kw = dict(directed=mode.get("directed", True), weight_tag=mode.get("weight_tag"), verbose=False,
              bidirected=mode.get("bidirected", False), keep_directed_bidir=mode.get("keep_directed_bidir", False),
              strip_orientation=False, dt=dt, asymmetric=mode.get("asymmetric", False), raw_bytes_id=False,
              return_node_list=True, device=0)
    return _parse_gfa_chunked(str(path), chunk, engine=CpuEngine(orc), **kw)


MODES = [{}, {"directed": False}, {"asymmetric": True}, {"dtype": "int8"}, {"dtype": "bool"}, {"dtype": "float32"}]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("chunk", [97, 1000, 7000, 1 << 30])
def test_chunked_equals_one_piece(oracle_lib, tmp_path, mode, chunk):
    from gfa2network_amd.api import finalize

    data = _decimal_gfa(21, 400, 2000)
    path = tmp_path / "in.gfa"
    path.write_bytes(data)
    got = _chunked(path, chunk, mode)
    assert got is not None
    A, nodes = got
    full = oracle_lib.run(data, **mode)
    B, bnodes = finalize(oracle_lib.to_raw(full, "parse"), dtype=np.dtype(mode.get("dtype", "float64")),
                         return_node_list=True, raw_bytes_id=False, verbose=False)
    assert A.format == B.format and A.shape == B.shape and A.dtype == B.dtype and nodes == bnodes
    if A.format == "coo":
        assert np.array_equal(A.row, B.row) and np.array_equal(A.col, B.col)
        assert A.row.dtype == B.row.dtype
    else:
        assert np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
        assert A.indptr.dtype == B.indptr.dtype
    assert A.data.tobytes() == B.data.tobytes()


@pytest.mark.parametrize("breaks", ["late_s", "ghost", "offset", "hashed", "error"])
def test_chunked_decimal_premise_breaks(oracle_lib, tmp_path, breaks):
    """A decimal-id premise break anywhere in the file — even one only the ranges' evidence together
    can see (an S line in a later range than an edge, names that start past 1, a key past the S
    count) — declines the decimal chunks (None); the merged-dictionary chunks then build the file
    (the one-piece answer), and a parse error declines both (the one-piece build raises it)."""
    from gfa2network_amd.api import finalize
    from gfa2network_amd.shard import _chunked_decimal
    from oracle import oracle as orc
    from shard_cpu_engine import CpuEngine

    data = _decimal_gfa(22, 300, 1200, breaks)
    path = tmp_path / "in.gfa"
    path.write_bytes(data)
    full = oracle_lib.run(data)
    for chunk in (113, 4000):
        assert _chunked_decimal(str(path), engine=CpuEngine(orc), chunk_bytes=chunk) is None, (breaks, chunk)
        got = _chunked(path, chunk, {})
        if breaks == "error":
            assert got is None
            continue
        A, nodes = got
        B, bnodes = finalize(oracle_lib.to_raw(full, "parse"), dtype=np.dtype("float64"), return_node_list=True,
                             raw_bytes_id=False, verbose=False)
        assert nodes == bnodes and np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)


@pytest.mark.parametrize("mode", [{"bidirected": True}, {"weight_tag": "RC"}])
def test_chunked_other_builds_take_the_general_chunks(oracle_lib, tmp_path, mode):
    """Bidirected / weighted decimal files are not the one-pass range parse's: the merged-dictionary
    chunks build them (same answer as one piece)."""
    from gfa2network_amd.api import finalize

    data = _decimal_gfa(23, 100, 300)
    path = tmp_path / "in.gfa"
    path.write_bytes(data)
    A, nodes = _chunked(path, 500, mode)
    full = oracle_lib.run(data, **mode)
    B, bnodes = finalize(oracle_lib.to_raw(full, "parse"), dtype=np.dtype("float64"), return_node_list=True,
                         raw_bytes_id=False, verbose=False)
    assert nodes == bnodes and A.data.tobytes() == B.data.tobytes()


def _named_gfa(seed, n_s, n_l, shuffle, extra=()):
    """Names that are not 1..N, edges before S lines, keys no S line defines, weights."""
    r = random.Random(seed)
    names = [f"s{k}" if k % 4 else f"node_{k:06d}_" + "q" * r.randint(0, 20) for k in range(n_s)]
    lines = [f"S\t{n}\t*\n" for n in names]
    for _ in range(n_l):
        a, b = r.choice(names), r.choice(names + ["ghost1", "ghost2"])
        lines.append(f"L\t{a}\t{r.choice('+-')}\t{b}\t{r.choice('+-')}\t*\tRC:i:{r.randint(0, 7)}\n")
    if shuffle:
        r.shuffle(lines)
    lines[len(lines) // 2:len(lines) // 2] = list(extra)
    return "".join(lines).encode()


GENERAL = [
    (False, {}), (True, {}), (True, {"directed": False}), (True, {"bidirected": True}),
    (True, {"bidirected": True, "keep_directed_bidir": True}), (True, {"asymmetric": True, "weight_tag": "RC",
                                                                     "dtype": "int32"}),
    (True, {"weight_tag": "RC", "dtype": "int8"}), (True, {"dtype": "bool"}),
    (True, {"weight_tag": "RC", "directed": False}), (False, {"weight_tag": "RC", "dtype": "float32"}),
]


@pytest.mark.parametrize("shuffle,mode", GENERAL)
@pytest.mark.parametrize("chunk", [211, 3000, 1 << 30])
def test_chunked_general_names_equal_one_piece(oracle_lib, tmp_path, shuffle, mode, chunk):
    """Any names: each chunk's keys merged into the file's dictionary in arrival order (the global
    first-touch ids), the chunk's triplets remapped — equal to the one-piece build, node list included."""
    from gfa2network_amd.api import finalize

    data = _named_gfa(31, 250, 1200, shuffle)
    path = tmp_path / "in.gfa"
    path.write_bytes(data)
    got = _chunked(path, chunk, mode)
    assert got is not None
    A, nodes = got
    full = oracle_lib.run(data, **mode)
    B, bnodes = finalize(oracle_lib.to_raw(full, "parse"), dtype=np.dtype(mode.get("dtype", "float64")),
                         return_node_list=True, raw_bytes_id=False, verbose=False)
    assert A.format == B.format and A.shape == B.shape and nodes == bnodes
    if A.format == "coo":
        assert np.array_equal(A.row, B.row) and np.array_equal(A.col, B.col)
    else:
        assert np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
    assert A.data.tobytes() == B.data.tobytes()


@pytest.mark.parametrize("extra", [["L\tbad\t+\n"], ["W\tsample\t1\tchr1\t0\t10\t>s1\n"]])
def test_chunked_general_declines_errors_and_warnings(oracle_lib, tmp_path, extra):
    path = tmp_path / "in.gfa"
    path.write_bytes(_named_gfa(32, 200, 800, True, extra))
    assert _chunked(path, 700, {}) is None


def test_auto_mode_chooses_chunks_only_past_free_memory(tmp_path, monkeypatch):
    """shard="auto" on one process: chunked only for a plain file on disk whose working set
    (WORKING_SET_PER_INPUT_BYTE x its size) passes the GPU's free HBM; never for "never"."""
    import torch

    from gfa2network_amd import api

    path = tmp_path / "in.gfa"
    path.write_bytes(_decimal_gfa(24, 50, 100))
    size = path.stat().st_size
    monkeypatch.setattr(api, "_dist_world", lambda: 1)
    for free, want in ((size * api.WORKING_SET_PER_INPUT_BYTE + 1, False), (size, True)):
        monkeypatch.setattr(torch.cuda, "mem_get_info", lambda device=None, f=free: (f, 2 * f))
        got = api._chunk_for(str(path), "auto", 0)
        assert bool(got) == want and (not got or got >= 1 << 26)
        assert api._chunk_for(str(path), "never", 0) == 0
    assert api._chunk_for(str(tmp_path / "missing.gfa"), "auto", 0) == 0
