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


def bgzf(data: bytes, block: int = 65280, level: int = 6, strategy: int = 0) -> bytes:
    """htslib's bgzip layout: members of at most 64 KiB of output, each with the 'BC' extra
    subfield holding its total size - 1, then the 28-byte EOF marker member."""
    import struct
    import zlib

    out = bytearray()
    for i in range(0, len(data), block):
        chunk = data[i:i + block]
        co = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
        cdata = co.compress(chunk) + co.flush()
        hdr = bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF]) + struct.pack("<H", 6) + b"BC" + struct.pack(
            "<HH", 2, 12 + 6 + len(cdata) + 8 - 1)
        out += hdr + cdata + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk))
    out += bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    return bytes(out)


@pytest.mark.parametrize("level,strategy", [(6, 0), (1, 0), (0, 0), (9, 1), (6, 2), (6, 3)])
def test_bgzf_inflated_on_gpu_equals_plain(gpu, tmp_path, monkeypatch, level, strategy):
    """A BGZF .gz (every deflate block kind: stored, fixed, dynamic; filtered / Huffman-only / RLE
    strategies) inflated on the GPU (g2n_inflate.hip: phase "gz_inflate") gives exactly the plain
    file's result, and the host readers (TEST_HOST_INFLATE) agree."""
    from gfa2network_amd import _native as nat
    from gfa2network_amd import parse_gfa, synth

    data = synth.host_bytes(60_000, 240_000, seed=11, rc_tag=True)
    plain, z = tmp_path / "p.gfa", tmp_path / "b.gfa.gz"
    plain.write_bytes(data)
    z.write_bytes(bgzf(data, level=level, strategy=strategy))
    raw = nat.build_from_path(str(z), nat.make_options())
    assert raw.status == 0 and "gz_inflate" in raw.phase_ms, sorted(raw.phase_ms)
    for mode in ({}, {"directed": False}, {"bidirected": True, "weight_tag": "RC"}):
        kw = dict(build_graph=False, build_matrix=True, return_node_list=True, **mode)
        want = _key(parse_gfa(plain, **kw))
        assert _key(parse_gfa(z, **kw)) == want, mode
        monkeypatch.setattr(nat, "TEST_FLAGS", nat.TEST_HOST_INFLATE)
        raw = nat.build_from_path(str(z), nat.make_options())
        assert "gz_inflate" not in raw.phase_ms
        assert _key(parse_gfa(z, **kw)) == want, mode
        monkeypatch.setattr(nat, "TEST_FLAGS", 0)


def test_bgzf_damaged_falls_back_to_exact_reader(gpu, tmp_path):
    """A BGZF chain whose members do not inflate cleanly (a bad CRC, a corrupt block, an
    incomplete code) goes to the host's gzip.py restatement: the same prefix parse and exception
    as a plain gzip.open loop."""
    import gzip
    import zlib

    from gfa2network_amd import parse_gfa, synth

    data = synth.host_bytes(20_000, 80_000, seed=12)
    good = bytearray(bgzf(data))
    cases = {}
    first_end = (good[16] | good[17] << 8) + 1  # member 1's size: its BC subfield + 1
    bad_crc = bytearray(good)
    bad_crc[first_end - 8] ^= 1  # member 1's CRC
    cases["crc"] = bytes(bad_crc)
    corrupt = bytearray(good)
    corrupt[first_end + 40:first_end + 60] = b"\xff" * 20  # inside member 2's deflate data
    cases["corrupt"] = bytes(corrupt)
    for name, blob in cases.items():
        p = tmp_path / f"{name}.gfa.gz"
        p.write_bytes(blob)
        try:
            for _ in gzip.open(p):
                pass
            want = None
        except (gzip.BadGzipFile, EOFError, zlib.error) as e:
            want = (type(e), str(e))
        with pytest.raises(Exception) as ei:
            parse_gfa(p, build_graph=False, build_matrix=True)
        assert want is not None and (type(ei.value), str(ei.value)) == want, name


@pytest.mark.parametrize("layout", ["zlib_level1", "pigz_pieces"])
def test_single_member_gzip_chunk_parallel(gpu, tmp_path, layout):
    """A single-member .gz of >= 64 MiB takes the chunk-parallel inflate (g2n_pinflate.cpp,
    SURVEY.md §8(f)2) inside g2n_build_from_path; the build equals the plain file's."""
    import gzip
    import sys
    from pathlib import Path

    from gfa2network_amd import _native, parse_gfa, synth

    data = synth.host_bytes(3_000_000, 12_000_000, seed=11)
    single = tmp_path / "s.gfa.gz"
    if layout == "zlib_level1":
        single.write_bytes(gzip.compress(data, 1, mtime=0))
    else:
        sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
        import bench

        bench.write_gz_single(data, str(single), level=6, threads=16, piece=16 << 20)
    blob = single.read_bytes()
    assert len(blob) >= 64 << 20, len(blob)
    got = _native.gunzip_chunked(blob)
    assert got is not None and got[1] > 1 and got[0] == data
    del got, blob
    kw = dict(build_graph=False, build_matrix=True, return_node_list=True, directed=False)
    want = _key(parse_gfa(io.BytesIO(data), **kw))
    assert _key(parse_gfa(single, **kw)) == want
