"""CPU: host-side result assembly (gfa2network_amd/api.py finalize) — no GPU."""
import numpy as np


def test_finalize_keeps_int64_index_arrays():
    """A native result in int64 indices (a coo.tocsr of more than 2^31 - 1 triplets: scipy sizes the
    index arrays by the COO's entries and keeps int64 after sum_duplicates) stays int64 — the
    csr_matrix constructor's content check alone would narrow small contents to int32."""
    from gfa2network_amd import _native as nat
    from gfa2network_amd.api import finalize

    raw = nat.RawResult(status=0, format="csr", n_nodes=3, dtype=np.dtype("float64"))
    raw.indptr = np.array([0, 1, 1, 2], dtype=np.int64)
    raw.indices = np.array([2, 0], dtype=np.int64)
    raw.data = np.array([1.0, 2.0])
    A = finalize(raw, dtype=np.dtype("float64"), return_node_list=False, raw_bytes_id=False, verbose=False)
    assert A.indptr.dtype == np.int64 and A.indices.dtype == np.int64
    assert A.toarray().tolist() == [[0, 0, 1.0], [0, 0, 0], [2.0, 0, 0]]
    raw.indptr, raw.indices = raw.indptr.astype(np.int32), raw.indices.astype(np.int32)
    B = finalize(raw, dtype=np.dtype("float64"), return_node_list=False, raw_bytes_id=False, verbose=False)
    assert B.indptr.dtype == np.int32
