"""dtypes outside the five the kernels compute in (VERDICT r05 "What's missing" 3), for unit-valued
builds: the build runs in int32 and its copy counts become the sum of that many ones in the dtype
(api._unit_values).  Checked here on the CPU against scipy's own arithmetic in that dtype
(builders.py:280-283: coo_matrix(data, dtype) then maximum(A.T); utils.py:55: tocsr), the copy
counts coming from scipy's int32 result of the same COO."""
import numpy as np
import pytest
import scipy.sparse as sp

EXTRA = ["int16", "int64", "uint8", "uint16", "uint32", "uint64", "longdouble", "complex64", "complex128"]


def _coo(seed, n=300, m=4000, dup=3):
    rng = np.random.default_rng(seed)
    r = rng.integers(0, n, m)
    c = (r + rng.geometric(0.3, m)) % n
    k = rng.integers(1, dup + 1, m)  # repeat some entries: copy counts > 1
    return np.repeat(r, k), np.repeat(c, k), n


@pytest.mark.parametrize("dt", EXTRA)
@pytest.mark.parametrize("seed", [0, 1])
def test_unit_values_equal_scipy_in_dtype(dt, seed):
    from gfa2network_amd.api import _with_unit_dtype

    r, c, n = _coo(seed)
    ones = [1.0] * len(r)  # builders.py:224-228 appends 1.0 without a weight tag
    # MAX-SYM (builders.py:282-283) and the SUM CSR (utils.py:55), each from the int32 build's counts
    want_ms = sp.coo_matrix((ones, (r, c)), shape=(n, n), dtype=np.dtype(dt))
    want_ms = want_ms.maximum(want_ms.T).tocsr()
    i32 = sp.coo_matrix((ones, (r, c)), shape=(n, n), dtype=np.int32)
    got_ms = _with_unit_dtype(i32.maximum(i32.T).tocsr(), np.dtype(dt), False)
    want_sum = sp.coo_matrix((ones, (r, c)), shape=(n, n), dtype=np.dtype(dt)).tocsr()
    got_sum = _with_unit_dtype(i32.tocsr(), np.dtype(dt), False)
    for got, want in ((got_ms, want_ms), (got_sum, want_sum)):
        assert got.dtype == want.dtype and got.indptr.dtype == want.indptr.dtype
        assert np.array_equal(got.indptr, want.indptr) and np.array_equal(got.indices, want.indices)
        assert np.array_equal(got.data, want.data)  # (longdouble: 80 bits in 16 bytes, padding undefined)
    # the COO result (directed=False / asymmetric): every value dtype(1.0)
    coo = _with_unit_dtype(i32, np.dtype(dt), False)
    want = sp.coo_matrix((ones, (r, c)), shape=(n, n), dtype=np.dtype(dt))
    assert coo.format == "coo" and coo.dtype == want.dtype and np.array_equal(coo.data, want.data)
    assert np.array_equal(coo.row, want.row) and np.array_equal(coo.col, want.col)


def test_unit_values_limits():
    from gfa2network_amd.api import _unit_values

    # sums that would wrap in the dtype: a documented limit, not a silent wrong value
    with pytest.raises(NotImplementedError):
        _unit_values(np.array([1, 256], dtype=np.int32), np.dtype("uint8"))
    with pytest.raises(NotImplementedError):
        _unit_values(np.array([32768], dtype=np.int32), np.dtype("int16"))
    assert _unit_values(np.array([255], dtype=np.int32), np.dtype("uint8")).tolist() == [255]
    # what scipy.sparse itself refuses, it refuses here too, with its own error
    with pytest.raises(ValueError, match="does not support dtype float16"):
        _unit_values(np.array([1], dtype=np.int32), np.dtype("float16"))
