"""CPU: the convert CLI's native writers against the reference's Python writers.

* save_npz (g2n_write_npz: zip64 members deflated on host threads) loads back through
  scipy.sparse.load_npz / numpy.load to exactly what scipy.sparse.save_npz stores (utils.py:85-86),
  for CSR / CSC / COO, every CLI dtype, empty matrices and members spanning many deflate pieces;
  the archive passes zipfile's CRC check.
* save_node_map_native (g2n_write_node_map) writes the bytes the reference's save_node_map
  (utils.py:108-114) writes, including the partial file and the UnicodeDecodeError of raw-bytes
  names that are not UTF-8.
"""
import random
import zipfile

import numpy as np
import pytest
import scipy.sparse as sp

from gfa2network_amd import _native
from gfa2network_amd.api import save_node_map, save_node_map_native, save_npz

DTYPES = ["bool", "int8", "int32", "float32", "float64"]


def _matrix(fmt, dtype, n, nnz, seed):
    r = np.random.default_rng(seed)
    rows = r.integers(0, max(n, 1), nnz)
    cols = r.integers(0, max(n, 1), nnz)
    data = (r.integers(1, 100, nnz)).astype(dtype)
    A = sp.coo_matrix((data, (rows, cols)), shape=(n, n), dtype=dtype)
    return A.asformat(fmt)


def _same(a, b):
    assert a.format == b.format and a.shape == b.shape and a.dtype == b.dtype
    for name in ("indptr", "indices", "row", "col", "data"):
        if hasattr(a, name):
            x, y = getattr(a, name), getattr(b, name)
            assert x.dtype == y.dtype and x.tobytes() == y.tobytes(), name


@pytest.mark.parametrize("fmt", ["csr", "csc", "coo"])
@pytest.mark.parametrize("dtype", DTYPES)
def test_npz_round_trip(tmp_path, fmt, dtype):
    for n, nnz in ((0, 0), (5, 0), (1000, 3000)):
        A = _matrix(fmt, dtype, n, nnz, hash((fmt, dtype, n)) & 0xFFFF)
        ours, ref = tmp_path / "a.npz", tmp_path / "b.npz"
        save_npz(ours, A)
        sp.save_npz(ref, A)
        _same(sp.load_npz(ours), sp.load_npz(ref))
        with np.load(ours) as x, np.load(ref) as y:
            assert x.files == y.files
            for k in x.files:
                assert x[k].dtype == y[k].dtype and x[k].shape == y[k].shape and x[k].tobytes() == y[k].tobytes()
        with zipfile.ZipFile(ours) as z:
            assert z.testzip() is None


def test_npz_many_pieces(tmp_path):
    A = _matrix("csr", "float64", 2_000_000, 3_000_000, 7)  # data 24 MB: several 8 MiB deflate pieces
    p = tmp_path / "big.npz"
    save_npz(p, A)
    _same(sp.load_npz(p), A)
    with zipfile.ZipFile(p) as z:
        assert z.testzip() is None
    save_npz(tmp_path / "noext", A)  # numpy appends the suffix
    _same(sp.load_npz(tmp_path / "noext.npz"), A)


def test_npz_unwritable_matches_scipy(tmp_path):
    A = _matrix("csr", "float64", 10, 20, 1)
    bad = tmp_path / "missing" / "x.npz"
    with pytest.raises(OSError) as e1:
        sp.save_npz(bad, A)
    with pytest.raises(OSError) as e2:
        save_npz(bad, A)
    assert type(e1.value) is type(e2.value) and str(e1.value) == str(e2.value)


def _blob(names):
    offs = np.zeros(len(names) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(x) for x in names])
    blob = np.frombuffer(b"".join(names) or b"\0", dtype=np.uint8)
    return blob, offs


def test_node_map_matches_reference_writer(tmp_path):
    r = random.Random(5)
    names = [str(i).encode() for i in range(1, 1_500_001)]
    names += ["ség☃".encode(), b"", b"x" * 300, "\U0001f600".encode()]
    r.shuffle(names)
    blob, offs = _blob(names)
    ours, ref = tmp_path / "a.tsv", tmp_path / "b.tsv"
    save_node_map_native(blob, offs, ours, raw_bytes_id=False)
    save_node_map([x.decode() for x in names], ref)
    assert ours.read_bytes() == ref.read_bytes()
    save_node_map_native(blob, offs, ours, raw_bytes_id=True)
    save_node_map(names, ref)
    assert ours.read_bytes() == ref.read_bytes()
    empty = _blob([])
    save_node_map_native(empty[0], empty[1], ours, raw_bytes_id=True)
    assert ours.read_bytes() == b""


@pytest.mark.parametrize("bad", [b"\xff", b"ab\xc3", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xc0\xaf", b"ok\xe2\x82"])
def test_node_map_raw_names_not_utf8(tmp_path, bad):
    names = [b"1", "é".encode(), b"3", bad, b"5"]
    blob, offs = _blob(names)
    assert _native.first_bad_utf8(blob, offs) == 3
    ours, ref = tmp_path / "a.tsv", tmp_path / "b.tsv"
    with pytest.raises(UnicodeDecodeError) as e1:
        save_node_map(names, ref)
    with pytest.raises(UnicodeDecodeError) as e2:
        save_node_map_native(blob, offs, ours, raw_bytes_id=True)
    assert str(e1.value) == str(e2.value)
    assert ours.read_bytes() == ref.read_bytes()
