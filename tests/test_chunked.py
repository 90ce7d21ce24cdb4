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
        if breaks == "error":  # the merged-dictionary chunks raise the one-piece build's error
            with pytest.raises(ValueError, match="Malformed L record"):
                _chunked(path, chunk, {})
            continue
        A, nodes = _chunked(path, chunk, {})
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


def _outcome(fn):
    """(kind, value, warnings): kind "ok" with (A, nodes), or "exc" with (type name, message)."""
    import warnings

    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        try:
            got = ("ok", fn())
        except Exception as e:  # noqa: BLE001 - compared against the one-piece build
            got = ("exc", (type(e).__name__, str(e)))
    return got[0], got[1], [str(x.message) for x in w]


def _one_piece(oracle_lib, data, mode):
    from gfa2network_amd.api import finalize

    def run():
        o = oracle_lib.run(data, **mode)
        return finalize(oracle_lib.to_raw(o, "parse"), dtype=np.dtype(mode.get("dtype", "float64")),
                        return_node_list=True, raw_bytes_id=False, verbose=False)
    return _outcome(run)


def _same(a, b):
    assert a[0] == b[0] and a[2] == b[2], (a[0], b[0], a[1] if a[0] == "exc" else "", b[1] if b[0] == "exc" else "",
                                           a[2], b[2])
    if a[0] == "exc":
        assert a[1] == b[1]
        return
    (A, na), (B, nb) = a[1], b[1]
    assert A.format == B.format and A.shape == B.shape and A.dtype == B.dtype and na == nb
    if A.format == "coo":
        assert np.array_equal(A.row, B.row) and np.array_equal(A.col, B.col) and A.row.dtype == B.row.dtype
    else:
        assert np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
        assert A.indptr.dtype == B.indptr.dtype
    assert A.data.tobytes() == B.data.tobytes()


ERRORS = {  # (text inserted near the middle of the file, mode): errors, cast errors and the warning
    "malformed_l": (["L\tbad\t+\n"], {}),
    "warning": (["W\tsample\t1\tchr1\t0\t10\t>s1\n"], {}),
    "two_warnings": (["W\tsample\t1\tchr1\t0\t10\t>s1\n", "J\tx\n"] * 3, {}),
    "warning_then_error": (["W\tsample\n"] + ["L\ts1\t+\ts2\t+\t*\n"] * 200 + ["L\tbad\n"], {}),
    "short_s": (["S\n"], {}),
    "cast_int8": (["L\ts1\t+\ts2\t+\t*\tRC:i:300\n"], {"weight_tag": "RC", "dtype": "int8"}),
    "cast_then_parse_error": (["L\ts1\t+\ts2\t+\t*\tRC:i:300\n"] + ["L\ts3\t+\ts1\t+\t*\n"] * 300
                              + ["L\tq\n"], {"weight_tag": "RC", "dtype": "int8"}),
    "float32_overflow": (["L\ts1\t+\ts2\t+\t*\tRC:i:" + "9" * 60 + "\n"], {"weight_tag": "RC", "dtype": "float32"}),
}


@pytest.mark.parametrize("case", sorted(ERRORS))
@pytest.mark.parametrize("chunk", [300, 2500, 1 << 30])
def test_chunked_errors_and_warnings_as_one_piece(oracle_lib, tmp_path, case, chunk):
    """Errors, cast errors and the one-shot unsupported-record warning anywhere in the file come out of
    the chunked build exactly as from one piece (parser.py:114-132, builders.py:281): the first parse
    error with its line (a cast error loses to a later parse error: the reference casts after its
    loop), one warning, float32 overflow warnings per element (GFA 1.1 W / J lines no longer
    send a large file to the one-piece build)."""
    extra, mode = ERRORS[case]
    data = _named_gfa(33, 150, 700, True, extra)
    path = tmp_path / "in.gfa"
    path.write_bytes(data)
    _same(_outcome(lambda: _chunked(path, chunk, mode)), _one_piece(oracle_lib, data, mode))


def _cpu_engine_factory(monkeypatch, oracle_mod, free=None):
    from gfa2network_amd import shard
    from shard_cpu_engine import CpuEngine

    def make(device=0, torch_buffers=True):
        e = CpuEngine(oracle_mod)
        if free is not None:
            e.free_bytes = free
        return e
    monkeypatch.setattr(shard, "HipEngine", make)


@pytest.mark.parametrize("kind", ["gz", "stdin", "fileobj", "plain"])
@pytest.mark.parametrize("mode", [{}, {"directed": False}, {"bidirected": True, "weight_tag": "RC"}])
def test_parse_gfa_chunks_every_input_kind(oracle_lib, tmp_path, monkeypatch, kind, mode):
    """parse_gfa itself (default shard="never") takes the one-GPU chunked build for an input past the
    GPU's working set, whatever its kind: a plain file (pread chunks), a .gz (inflated on the host, then
    chunked from host memory), stdin and a file object (read, then chunked) — equal to one piece.  Here
    the GPU's free HBM is reported small and the CPU engine stands in for the HIP one."""
    import gzip
    import io
    import sys

    from gfa2network_amd import api, parse_gfa

    data = _named_gfa(34, 200, 900, True)
    _cpu_engine_factory(monkeypatch, __import__("oracle.oracle", fromlist=["x"]))
    monkeypatch.setattr(api, "_free_hbm", lambda device=0, need=0: 1000)  # every input is past the working set
    monkeypatch.setattr(api, "_chunk_plan", lambda size, device: 1500 if size * 8 > 1000 else 0)
    calls = []
    real = api._parse_gfa_chunked
    monkeypatch.setattr(api, "_parse_gfa_chunked", lambda *a, **k: calls.append(1) or real(*a, **k))
    if kind == "gz":
        src = tmp_path / "in.gfa.gz"
        src.write_bytes(gzip.compress(data[:len(data) // 2]) + gzip.compress(data[len(data) // 2:]))
    elif kind == "plain":
        src = tmp_path / "in.gfa"
        src.write_bytes(data)
    elif kind == "fileobj":
        src = io.BytesIO(data)
    else:
        src = "-"
        monkeypatch.setattr(sys, "stdin", type("S", (), {"buffer": io.BytesIO(data)})())
    got = _outcome(lambda: parse_gfa(src, build_graph=False, build_matrix=True, return_node_list=True, **mode))
    assert calls, "the chunked build did not run"
    _same(got, _one_piece(oracle_lib, data, mode))


@pytest.mark.parametrize("mode", [{}, {"directed": False}, {"dtype": "int8"},
                                  {"weight_tag": "RC", "dtype": "float32"}, {"weight_tag": "RC", "asymmetric": True},
                                  {"bidirected": True}])
@pytest.mark.parametrize("bands", [2, 5])
def test_chunked_csr_in_row_bands_equals_one_piece(oracle_lib, tmp_path, mode, bands):
    """The whole-matrix CSR of a chunked build assembled in row bands (each chunk's triplets routed by
    band, stable; each band's CSR with its row base; indptrs rebased) equals one piece — the path a
    file takes when its CSR does not fit the GPU beside its triplets (floats: scipy's whole-matrix
    has_sorted_indices verdict OR-ed over the bands first)."""
    from gfa2network_amd.api import _dtype_of, _parse_gfa_chunked
    from oracle import oracle as orc
    from shard_cpu_engine import CpuEngine

    data = _named_gfa(35, 120, 900, True)
    path = tmp_path / "in.gfa"
    path.write_bytes(data)
    kw = dict(directed=mode.get("directed", True), weight_tag=mode.get("weight_tag"), verbose=False,
              bidirected=mode.get("bidirected", False), keep_directed_bidir=False, strip_orientation=False,
              dt=_dtype_of(mode.get("dtype", "float64")), asymmetric=mode.get("asymmetric", False),
              raw_bytes_id=False, return_node_list=True, device=0)
    got = _outcome(lambda: _parse_gfa_chunked(str(path), 900, engine=CpuEngine(orc), bands=bands, **kw))
    _same(got, _one_piece(oracle_lib, data, mode))


def test_chunked_assembly_sizes_bands_from_free_memory(oracle_lib, tmp_path):
    """With the GPU's free HBM below the whole CSR's estimate the assembly picks row bands by itself
    (equal to one piece); below even the band-ordered triplets it raises MemoryError (ADVICE r04:
    a clear error instead of running out of device memory part way)."""
    from gfa2network_amd import shard
    from gfa2network_amd.api import _dtype_of, _parse_gfa_chunked
    from oracle import oracle as orc
    from shard_cpu_engine import CpuEngine

    data = _decimal_gfa(36, 300, 3000)
    path = tmp_path / "in.gfa"
    path.write_bytes(data)
    kw = dict(directed=True, weight_tag=None, verbose=False, bidirected=False, keep_directed_bidir=False,
              strip_orientation=False, dt=_dtype_of("float64"), asymmetric=False, raw_bytes_id=False,
              return_node_list=True, device=0)
    n_trip = 3000
    whole = shard.csr_bytes_estimate(n_trip, n_trip, 300, 8) + 16 * n_trip
    seen = {}
    real = shard._assemble_csr

    def spy(*a, **k):
        out = real(*a, **k)
        seen["bands"] = a[6].get("csr_bands", 1)
        return out
    shard._assemble_csr = spy
    try:
        eng = CpuEngine(orc)
        eng.free_bytes = whole // 2
        got = _outcome(lambda: _parse_gfa_chunked(str(path), 5000, engine=eng, **kw))
        _same(got, _one_piece(oracle_lib, data, {}))
        assert seen["bands"] >= 2
        eng.free_bytes = 1000
        with pytest.raises(MemoryError, match="needs about"):
            _parse_gfa_chunked(str(path), 5000, engine=eng, **kw)
    finally:
        shard._assemble_csr = real


def test_chunk_plan_only_past_free_memory(tmp_path, monkeypatch):
    """The one-GPU chunked build starts only for an input whose working set (WORKING_SET_PER_INPUT_BYTE
    x its size) passes the GPU's free HBM, read through the C-ABI (no torch); without a device no chunks
    (the build raises the device error)."""
    from gfa2network_amd import api

    size = 10 << 20
    for free, want in ((size * api.WORKING_SET_PER_INPUT_BYTE + 1, False), (size, True)):
        monkeypatch.setattr(api, "_free_hbm", lambda device=0, need=0, f=free: f)
        got = api._chunk_plan(size, 0)
        assert bool(got) == want and (not got or got >= 1 << 26)
    monkeypatch.setattr(api, "_free_hbm", lambda device=0, need=0: None)
    assert api._chunk_plan(size, 0) == 0


def test_line_ranges_windowed_search():
    """line_ranges over a host buffer finds each boundary without scanning past the next newline
    (a chunked .gz / stdin input may be hundreds of GB); long lines and missing newlines kept."""
    from gfa2network_amd.shard import line_ranges

    r = __import__("random").Random(5)
    for _ in range(50):
        parts = [b"x" * r.choice([0, 1, 5, 70000, 200000]) + b"\n" for _ in range(r.randint(0, 12))]
        data = b"".join(parts) + (b"tail" if r.random() < 0.5 else b"")
        arr = np.frombuffer(data, dtype=np.uint8)
        n = r.randint(1, 9)
        got = line_ranges(arr, n)
        want, starts = [], [0]
        for k in range(1, n):
            s = k * len(data) // n
            if 0 < s < len(data) and data[s - 1] != 0x0A:
                j = data.find(b"\n", s)
                s = len(data) if j < 0 else j + 1
            starts.append(max(s, starts[-1]))
        want = [(starts[k], starts[k + 1] if k + 1 < n else len(data)) for k in range(n)]
        assert got == want
