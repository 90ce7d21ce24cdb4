"""GPU: the host ingest of g2n_build_from_path (pinned staged H2D in 16 MiB slots, parallel
multi-member gunzip) hands the pipeline exactly the bytes the buffer entry point does, on inputs
spanning many staging slots and gzip members; and the results equal the oracle."""
import io

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _members(data: bytes, size: int) -> bytes:
    import gzip

    return b"".join(gzip.compress(data[i:i + size], 1, mtime=0) for i in range(0, len(data), size))


def _key(res):
    A, nodes = res
    arrs = (A.indptr, A.indices, A.data) if A.format == "csr" else (A.row, A.col, A.data)
    return (A.format, A.shape, str(A.dtype), tuple(a.tobytes() for a in arrs), nodes)


@pytest.mark.parametrize("mode", [{}, {"directed": False}, {"bidirected": True, "weight_tag": "RC"}])
def test_path_ingest_equals_buffer(gpu, tmp_path, mode):
    import gzip

    from gfa2network_amd import parse_gfa, synth

    data = synth.host_bytes(1_000_000, 4_000_000, seed=5, rc_tag="weight_tag" in mode)
    assert len(data) > 6 * (16 << 20)  # several staging slots
    kw = dict(build_graph=False, build_matrix=True, return_node_list=True, **mode)
    want = _key(parse_gfa(io.BytesIO(data), **kw))
    plain = tmp_path / "x.gfa"
    plain.write_bytes(data)
    assert _key(parse_gfa(plain, **kw)) == want
    multi = tmp_path / "m.gfa.gz"
    multi.write_bytes(_members(data, 5 << 20) + b"\0\0")
    assert _key(parse_gfa(multi, **kw)) == want
    if not mode:
        single = tmp_path / "s.gfa.gz"
        single.write_bytes(gzip.compress(data, 1, mtime=0))
        assert _key(parse_gfa(single, **kw)) == want


def test_path_ingest_equals_oracle(gpu, oracle_lib, tmp_path):
    from gfa2network_amd import convert_format, parse_gfa, synth
    from gfa2network_amd.api import finalize

    data = synth.host_bytes(200_000, 800_000, seed=9)
    p = tmp_path / "y.gfa.gz"
    p.write_bytes(_members(data, 3 << 20))
    A, nodes = parse_gfa(p, build_graph=False, build_matrix=True, return_node_list=True, directed=False)
    o = oracle_lib.run(data, directed=False)
    B, onodes = finalize(oracle_lib.to_raw(o, "parse"), dtype=np.dtype("float64"), return_node_list=True,
                         raw_bytes_id=False, verbose=False)
    assert nodes == onodes
    assert A.row.tobytes() == B.row.tobytes() and A.col.tobytes() == B.col.tobytes()
    assert A.data.tobytes() == B.data.tobytes()
    C, R = convert_format(A, "csr"), oracle_lib.to_raw(o, "csr")
    assert C.indptr.tobytes() == R.indptr.tobytes() and C.indices.tobytes() == R.indices.tobytes()
    assert C.data.tobytes() == R.data.tobytes()
