"""One file built on one GPU in line-aligned chunks (shard.build_chunked, parse_gfa's chunked mode)
equals the one-piece build — here on the CPU engine (the oracle per range, scipy for the CSR), on
the HIP engine in test_gpu_shard.py.  Chunk sizes from 97 bytes (dozens of ranges, S sections and
edge sections split anywhere) to the whole file; every premise break declines (None) so the caller
builds in one piece."""
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
def test_chunked_declines_when_the_premise_breaks(oracle_lib, tmp_path, breaks):
    """A premise break anywhere in the file — even one only the ranges' evidence together can see
    (an S line in a later range than an edge, names that start past 1, a key past the S count) — or
    a parse error declines: the one-piece build then decides (and raises the reference's error)."""
    data = _decimal_gfa(22, 300, 1200, breaks)
    path = tmp_path / "in.gfa"
    path.write_bytes(data)
    for chunk in (113, 4000):
        assert _chunked(path, chunk, {}) is None, (breaks, chunk)


@pytest.mark.parametrize("mode", [{"bidirected": True}, {"weight_tag": "RC"}])
def test_chunked_declines_other_builds(oracle_lib, tmp_path, mode):
    path = tmp_path / "in.gfa"
    path.write_bytes(_decimal_gfa(23, 100, 300))
    assert _chunked(path, 500, mode) is None
