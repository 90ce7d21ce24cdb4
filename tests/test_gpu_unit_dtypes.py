"""parse_gfa / convert_format in dtypes outside the five the kernels compute in (unit values: no weight
tag), on the GPU, against the reference's own arithmetic: scipy in that dtype on the oracle's
stream-order COO (builders.py:279-283: coo_matrix((data, (rows, cols)), dtype) and maximum(A.T);
utils.py:55: tocsr / tocsc) — values, index arrays, dtypes and the node list."""
import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu

EXTRA = ["int16", "int64", "uint8", "uint16", "uint32", "uint64", "longdouble", "complex128"]


def _input():
    from gfa2network_amd import synth

    base = synth.host_bytes(20_000, 80_000, seed=7)
    # repeated L lines: copy counts above 1 in both directions
    extra = b"".join(b"L\t%d\t+\t%d\t-\t*\n" % (a, a + 1) for a in range(1, 400)) * 3
    return base + extra


def _want(oracle_lib, data, dt, directed):
    from oracle import oracle as orc

    full = orc.run(data, directed=directed)
    n = full.n_nodes
    A = sp.coo_matrix(([1.0] * len(full.rows), (full.rows, full.cols)), shape=(n, n), dtype=np.dtype(dt))
    names = [bytes(full.names_blob[full.names_offsets[i]:full.names_offsets[i + 1]]).decode() for i in range(n)]
    return (A.maximum(A.T) if directed else A), names


@pytest.mark.parametrize("dt", EXTRA)
def test_parse_gfa_unit_dtypes_equal_scipy(gpu, oracle_lib, tmp_path, dt):
    from gfa2network_amd import convert_format, parse_gfa

    data = _input()
    path = tmp_path / "g.gfa"
    path.write_bytes(data)
    for directed in (True, False):
        A, nodes = parse_gfa(str(path), build_graph=False, build_matrix=True, directed=directed, dtype=dt,
                             return_node_list=True)
        W, want_nodes = _want(oracle_lib, data, dt, directed)
        assert nodes == want_nodes and A.dtype == W.dtype and A.format == W.format, (dt, directed)
        if directed:  # MAX-SYM CSR
            assert np.array_equal(A.indptr, W.indptr) and np.array_equal(A.indices, W.indices)
            assert A.indptr.dtype == W.indptr.dtype and np.array_equal(A.data, W.data)
        else:  # the stream-order COO, then convert --undirected (coo.tocsr / tocsc)
            assert np.array_equal(A.row, W.row) and np.array_equal(A.col, W.col) and np.array_equal(A.data, W.data)
            for fmt in ("csr", "csc"):
                C, WC = convert_format(A, fmt), W.asformat(fmt)
                assert C.dtype == WC.dtype and C.indptr.dtype == WC.indptr.dtype, (dt, fmt)
                assert np.array_equal(C.indptr, WC.indptr) and np.array_equal(C.indices, WC.indices)
                assert np.array_equal(C.data, WC.data), (dt, fmt)


def test_parse_gfa_unit_dtype_refusals(gpu, tmp_path):
    from gfa2network_amd import convert_format, parse_gfa

    path = tmp_path / "g.gfa"
    path.write_bytes(b"S\t1\t*\nS\t2\t*\n" + b"L\t1\t+\t2\t+\t*\tRC:i:3\n" * 300)
    # a weight tag in another dtype: not on the GPU path
    with pytest.raises(NotImplementedError):
        parse_gfa(str(path), build_graph=False, build_matrix=True, dtype="int64", weight_tag="RC")
    # 300 copies of one entry wrap in uint8: a documented limit, never a wrapped value
    with pytest.raises(NotImplementedError):
        parse_gfa(str(path), build_graph=False, build_matrix=True, dtype="uint8")
    assert parse_gfa(str(path), build_graph=False, build_matrix=True, dtype="uint16").data.tolist() == [300, 300]
    # scipy.sparse refuses float16 itself (so does the reference at builders.py:280)
    with pytest.raises(ValueError, match="float16"):
        parse_gfa(str(path), build_graph=False, build_matrix=True, dtype="float16")
    # convert_format of another dtype with values other than 1: not on the GPU path
    A = sp.coo_matrix((np.array([2, 1], dtype=np.int64), ([0, 1], [1, 0])), shape=(2, 2))
    with pytest.raises(NotImplementedError):
        convert_format(A, "csr")
