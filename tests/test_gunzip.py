"""CPU: the library's gzip reader (g2n_gunzip — what g2n_build_from_path runs for ".gz" names,
parser.py:108-109 gzip.open) against CPython's gzip module on the same bytes: identical output,
or the identical exception type and message.  Both the parallel member path and the serial
reader are checked; no GPU is needed (inflate is host work)."""
from __future__ import annotations

import gzip
import io
import random
import struct
import zlib

import pytest

from gfa2network_amd import _native

EXC = {1: gzip.BadGzipFile, 2: EOFError, 3: zlib.error, 4: gzip.BadGzipFile}


def member(data: bytes, level: int = 6, flags: int = 0, extra: bytes = b"", name: bytes = b"",
           comment: bytes = b"", hcrc: int | None = None, method: int = 8) -> bytes:
    """One gzip member with the requested optional header fields (RFC 1952)."""
    hdr = bytearray(b"\x1f\x8b" + bytes([method, flags]) + struct.pack("<I", 0) + b"\x00\xff")
    if flags & 4:
        hdr += struct.pack("<H", len(extra)) + extra
    if flags & 8:
        hdr += name + b"\x00"
    if flags & 16:
        hdr += comment + b"\x00"
    if flags & 2:
        hdr += struct.pack("<H", (zlib.crc32(hdr) & 0xFFFF) if hcrc is None else hcrc)
    co = zlib.compressobj(level, zlib.DEFLATED, -zlib.MAX_WBITS)
    body = co.compress(data) + co.flush()
    return bytes(hdr) + body + struct.pack("<II", zlib.crc32(data), len(data) & 0xFFFFFFFF)


def gfa_text(n: int, seed: int) -> bytes:
    r = random.Random(seed)
    lines = [f"S\t{i}\t{''.join(r.choice('ACGT') for _ in range(r.randint(0, 30)))}" for i in range(1, n + 1)]
    lines += [f"L\t{r.randint(1, n)}\t+\t{r.randint(1, n)}\t-\t0M" for _ in range(2 * n)]
    return ("\n".join(lines) + "\n").encode()


def python_read(blob: bytes):
    try:
        return gzip.GzipFile(fileobj=io.BytesIO(blob)).read(), None
    except (gzip.BadGzipFile, EOFError, zlib.error) as e:
        return None, e


def python_lines_before_error(blob: bytes) -> bytes:
    """The lines parser.py:114's `for line in fh` sees on gzip.open before the exception."""
    seen = []
    try:
        for line in gzip.GzipFile(fileobj=io.BytesIO(blob)):
            seen.append(line)
    except (gzip.BadGzipFile, EOFError, zlib.error):
        pass
    return b"".join(seen)


def check(blob: bytes, members: int | None = None):
    want, exc = python_read(blob)
    for parallel in (True, False):
        if exc is None:
            got, m = _native.gunzip(blob, parallel=parallel)
            assert got == want
            if members is not None:
                assert m == members
        else:
            with pytest.raises(_native.GzipFailure) as ei:
                _native.gunzip(blob, parallel=parallel)
            f = ei.value
            assert EXC[f.sub] is type(exc), (f.sub, f.message, exc)
            assert f.message == str(exc)
            # the whole lines of what the reader returned first (the prefix g2n_build_from_path
            # parses before raising the gzip error)
            cut = f.prefix.rfind(b"\n") + 1
            assert f.prefix[:cut] == python_lines_before_error(blob), (f.sub, f.message)


T = gfa_text(3000, 1)
PARTS = [T[: len(T) // 3], T[len(T) // 3: 2 * len(T) // 3], T[2 * len(T) // 3:]]


def test_empty_and_single():
    check(b"", 0)
    check(member(b""), 1)
    check(member(T), 1)
    check(member(T, level=0), 1)
    check(member(T, level=9), 1)


def test_multi_member_and_padding():
    check(b"".join(member(p) for p in PARTS), 3)
    check(member(PARTS[0]) + b"\x00" * 7 + member(PARTS[1]) + b"\x00" * 3, 2)
    check(b"".join(member(T[i:i + 997]) for i in range(0, len(T), 997)))


def test_header_fields():
    check(member(T, flags=4, extra=b"BC\x02\x00\x00\x00"), 1)
    check(member(T, flags=8, name=b"x.gfa") + member(T, flags=16, comment=b"hello"), 2)
    check(member(T, flags=2 | 4 | 8 | 16, extra=b"ab", name=b"n", comment=b"c"), 1)
    check(member(T, flags=2, hcrc=0x1234))  # wrong header CRC: gzip.py never checks it
    check(member(T, flags=0x20))  # reserved flag bit: gzip.py ignores it, zlib would not


def test_errors_match_gzip_module():
    good = member(T)
    check(b"\x00\x00" + good)  # leading zeros are not padding
    check(good + b"xy")  # trailing garbage
    check(good + b"x")  # a single trailing byte
    check(good + b"\x00\x00x\x00")  # garbage after padding
    check(b"\x1f")
    check(b"ab")
    check(good[:5])  # truncated header
    check(good[: len(good) // 2])  # truncated deflate data
    check(good[:-3])  # truncated trailer
    check(member(T, method=7))
    bad = bytearray(good)
    bad[len(bad) // 2] ^= 0xFF
    check(bytes(bad))  # corrupt deflate data (or a CRC error, whichever zlib meets)
    crc = bytearray(good)
    crc[-8] ^= 1
    check(bytes(crc))
    ln = bytearray(good)
    ln[-1] ^= 1
    check(bytes(ln))
    check(member(T, flags=4, extra=b"abc")[:12])


def test_embedded_gzip_is_not_a_member():
    # a stored (level 0) member whose payload is itself a gzip file: its inner header is a member
    # candidate that inflates cleanly, yet it is not on the member chain
    inner = member(T) + member(PARTS[0])
    check(member(inner, level=0) + member(PARTS[1]), 2)


@pytest.mark.parametrize("seed", range(8))
def test_random_member_chains(seed):
    r = random.Random(seed)
    text = gfa_text(r.randint(100, 2000), seed) + bytes(r.randrange(256) for _ in range(200))
    cuts = sorted(r.sample(range(1, len(text)), r.randint(0, 12)))
    pieces = [text[a:b] for a, b in zip([0] + cuts, cuts + [len(text)])]
    blob = b"".join(member(p, level=r.choice([0, 1, 6, 9])) + b"\x00" * r.choice([0, 0, 1, 5]) for p in pieces)
    check(blob, len(pieces))
    if r.random() < 0.5:
        cut = r.randrange(len(blob))
        check(blob[:cut])


def stored_block_headers(m: bytes, hdr_len: int = 10) -> list[int]:
    """Offsets of the stored-block headers of a level-0 member (RFC 1951 3.2.4: one byte of
    BFINAL / BTYPE = 00 bits, then LEN, NLEN; the block's bytes follow)."""
    pos, out = hdr_len, []
    while True:
        out.append(pos)
        final = m[pos] & 1
        ln = m[pos + 1] | (m[pos + 2] << 8)
        pos += 5 + ln
        if final:
            return out


@pytest.mark.parametrize("seed", range(4))
def test_corrupt_deflate_prefix_follows_8k_refills(seed):
    """zlib.error mid-member: gzip.py discards the output of the failing decompress call, whose
    input and output windows follow io.BufferedReader's 8192-byte refills — the prefix the
    library reports is exactly the lines a line loop saw.  Stored blocks with a broken NLEN
    ("invalid stored block lengths") put the error at every block of the member in turn;
    random overwrites of compressed members and truncations add the other error kinds."""
    r = random.Random(100 + seed)
    text = gfa_text(r.randint(3000, 9000), seed)
    m0 = member(text, level=0)
    n_zlib = 0
    for at in stored_block_headers(m0):
        bad = bytearray(m0)
        bad[at + 3] ^= 0x5A  # NLEN no longer ~LEN
        n_zlib += python_read(bytes(bad))[1].__class__ is zlib.error
        check(bytes(bad))
    assert n_zlib >= 2
    m = member(text, level=r.choice([1, 6, 9]))
    for _ in range(12):
        bad = bytearray(m)
        at = r.randrange(12, len(bad) - 8)
        k = r.randint(4, 64)
        bad[at:at + k] = bytes(r.randrange(256) for _ in range(len(bad[at:at + k])))
        check(bytes(bad))
        check(m[:at])  # truncated there


# ---- chunk-parallel single-member inflate (g2n_pinflate.cpp) -------------
def _single_member_pieces(data: bytes, piece: int, level: int = 6) -> bytes:
    """pigz-style ONE member: pieces primed with the 32 KiB before them, sync-flushed."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench

    import tempfile
    with tempfile.NamedTemporaryFile(suffix=".gz") as fh:
        bench.write_gz_single(data, fh.name, level=level, threads=4, piece=piece)
        return Path(fh.name).read_bytes()


@pytest.fixture(scope="module")
def big_text() -> bytes:
    return gfa_text(60_000, 7) * 2


@pytest.mark.parametrize("level", [1, 6, 9])
@pytest.mark.parametrize("strategy", [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE])
@pytest.mark.parametrize("chunk", [1 << 16, 1 << 18, 0])
def test_chunked_equals_zlib(big_text, level, strategy, chunk):
    co = zlib.compressobj(level, zlib.DEFLATED, 31, 8, strategy)
    blob = co.compress(big_text) + co.flush()
    got = _native.gunzip_chunked(blob, chunk)
    assert got is not None, "a zlib single member with dynamic blocks must be taken"
    assert got[0] == big_text
    if chunk and chunk < len(blob) // 4:
        assert got[1] > 1, "more than one chunk must decode from a block start of its own"


def test_chunked_fixed_and_stored_blocks(big_text):
    # fixed-Huffman-only and stored-only streams: no dynamic block start to sync on, so the
    # first chunk decodes everything; the result is still exact
    for co in (zlib.compressobj(6, zlib.DEFLATED, 31, 8, zlib.Z_FIXED), zlib.compressobj(0, zlib.DEFLATED, 31)):
        blob = co.compress(big_text[:400_000]) + co.flush()
        got = _native.gunzip_chunked(blob, 1 << 14)
        assert got is not None and got[0] == big_text[:400_000] and got[1] == 1


def test_chunked_pigz_layout_and_mixed_blocks(big_text):
    blob = _single_member_pieces(big_text, piece=300_000)
    assert gzip.decompress(blob) == big_text
    got = _native.gunzip_chunked(blob, 1 << 16)
    assert got is not None and got[0] == big_text and got[1] > 1
    # incompressible stretches (stored blocks) between text
    r = random.Random(3)
    mixed = b"".join(big_text[i:i + 200_000] + bytes(r.getrandbits(8) for _ in range(70_000))
                     for i in range(0, 1_000_000, 200_000))
    blob = gzip.compress(mixed, 6)
    got = _native.gunzip_chunked(blob, 1 << 15)
    assert got is not None and got[0] == mixed


@pytest.mark.parametrize("damage", ["trailing_member", "trailing_garbage", "truncated", "crc", "isize",
                                    "bitflip", "zero_padding"])
def test_chunked_declines_or_matches(big_text, damage):
    blob = bytearray(gzip.compress(big_text, 6))
    if damage == "trailing_member":
        blob += gzip.compress(b"S\t1\n")
    elif damage == "trailing_garbage":
        blob += b"garbage"
    elif damage == "truncated":
        del blob[len(blob) // 2:]
    elif damage == "crc":
        blob[-8] ^= 1
    elif damage == "isize":
        blob[-4] ^= 1
    elif damage == "bitflip":
        blob[len(blob) // 3] ^= 0x10
    elif damage == "zero_padding":
        blob += b"\x00" * 100
    blob = bytes(blob)
    got = _native.gunzip_chunked(blob, 1 << 16)
    want, err = python_read(blob)
    if damage == "zero_padding":
        assert got is not None and got[0] == want
    elif got is not None:
        # taken only when gzip.py reads exactly one clean member to the end
        assert err is None and got[0] == want
    else:
        assert damage != "zero_padding"
    # the full reader (which tries the chunked path first on big files) stays exact
    for parallel in (True, False):
        try:
            out, _ = _native.gunzip(blob, parallel=parallel)
            assert err is None and out == want
        except _native.GzipFailure as e:
            assert err is not None and isinstance(err, EXC[e.sub]) and e.message == str(err)


def test_chunked_reference_before_stream_start():
    # a stream whose first chunk is shorter than the window the next chunk reads from: a
    # back-reference before the stream's first byte must never be filled from nowhere
    text = b"ACGT" * 5 + gfa_text(3000, 1)
    blob = gzip.compress(text, 9)
    for chunk in (64, 256, 1024):
        got = _native.gunzip_chunked(blob, chunk)
        assert got is None or got[0] == text
