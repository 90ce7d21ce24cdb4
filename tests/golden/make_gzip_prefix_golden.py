#!/usr/bin/env python3
"""Golden fixtures for corrupt / truncated ``.gz`` inputs, from the REAL reference.

The reference streams a ``.gz`` input (parser.py:108-114: ``for line in gzip.open(path)``): the
lines gzip returns before a failure are parsed — their parse error wins, their unsupported-record
warning and verbose progress come first — and then the gzip exception propagates.  The export
command (cli.py:264-281) writes those lines' edges before raising.

Runs ONLY in the build container, where the pure-Python reference is importable from
/root/reference.  Writes the inputs to tests/golden/inputs_gz/ and, per input,
``parse_gfa(path, build_graph=False, build_matrix=True, return_node_list=True, **mode)``'s
exception / warnings / verbose stderr and ``cli.main(["export", ...])``'s bytes written /
exception / warnings to tests/golden/expected/gzip_prefix.json (plain data).
"""
from __future__ import annotations

import base64
import contextlib
import gzip
import hashlib
import io
import json
import struct
import sys
import tempfile
import warnings
import zlib
from pathlib import Path

REF = "/root/reference"
HERE = Path(__file__).resolve().parent
INPUTS = HERE / "inputs_gz"
MODES = {"default": {}, "undirected_int8": {"directed": False, "dtype": "int8"},
         "bidir_rc": {"bidirected": True, "weight_tag": "RC"}}


def member(data: bytes, level: int = 6) -> bytes:
    co = zlib.compressobj(level, zlib.DEFLATED, -zlib.MAX_WBITS)
    body = co.compress(data) + co.flush()
    hdr = b"\x1f\x8b\x08\x00" + struct.pack("<I", 0) + b"\x00\xff"
    return hdr + body + struct.pack("<II", zlib.crc32(data), len(data) & 0xFFFFFFFF)


def gfa(n: int, extra: dict[int, str] | None = None) -> bytes:
    """n S lines then 3n L lines (RC tags), with `extra` lines inserted before line index k."""
    lines = [f"S\t{i}\t{'ACGT' * (i % 5)}" for i in range(1, n + 1)]
    lines += [f"L\t{1 + (7 * k) % n}\t{'+-'[k % 2]}\t{1 + (13 * k + 5) % n}\t{'-+'[k % 3 == 0]}\t0M\tRC:i:{k % 9}"
              for k in range(3 * n)]
    for k, line in sorted((extra or {}).items(), reverse=True):
        lines.insert(k, line)
    return ("\n".join(lines) + "\n").encode()


def stored_member(data: bytes, sizes: list[int]) -> bytes:
    """A member of stored deflate blocks (RFC 1951 3.2.4) of the given sizes, then the rest."""
    body, pos = bytearray(), 0
    cuts = []
    for n in sizes:
        cuts.append(min(pos + n, len(data)))
        pos = cuts[-1]
    while pos < len(data):
        pos = min(pos + 60000, len(data))
        cuts.append(pos)
    prev = 0
    for i, c in enumerate(cuts):
        ln = c - prev
        body += bytes([1 if i == len(cuts) - 1 else 0]) + struct.pack("<HH", ln, ln ^ 0xFFFF) + data[prev:c]
        prev = c
    hdr = b"\x1f\x8b\x08\x00" + struct.pack("<I", 0) + b"\x00\xff"
    return hdr + bytes(body) + struct.pack("<II", zlib.crc32(data), len(data) & 0xFFFFFFFF)


def inputs() -> dict[str, bytes]:
    out = {}
    m = member(gfa(300, {40: "L\t1\t+"}))
    out["trunc_malformed_early"] = m[: int(len(m) * 0.7)]
    m = member(gfa(300, {10: "X\tunknown\trecord"}))
    out["trunc_unknown"] = m[: int(len(m) * 0.6)]
    m = member(gfa(300))
    out["trunc_clean"] = m[: int(len(m) * 0.5)]
    big = b"S\t1\t*\nS\t2\t*\n" + b"L\t1\t+\t2\t-\t0M\n" * 600_000
    m = member(big, level=9)
    out["trunc_verbose"] = m[:-40]
    m = bytearray(member(gfa(300, {1199: "L\t2\t-\t3"})))
    m[-8] ^= 1
    out["crc_malformed_late"] = bytes(m)
    m = bytearray(member(gfa(300, {5: "Z\tz"})))
    m[-8] ^= 1
    out["crc_unknown"] = bytes(m)
    out["garbage_tail_unknown"] = member(gfa(200, {7: "Q\tq"})) + b"XY"
    out["garbage_tail_malformed"] = member(gfa(200, {790: "C\t1"})) + b"\x1f\x8bXX"
    # stored blocks of chosen sizes, block 1's NLEN broken: the call that meets it is gzip.py's
    # 4th 8192-byte refill, which also held block 0's last 5430 bytes — a malformed line in those
    # is lost with that call's output (zlib.error wins), one before them is parsed (ValueError)
    text = gfa(800)
    for back in (100, 3000, 5000, 6000, 9000):
        k = text.count(b"\n", 0, 30001 - back)
        t2 = gfa(800, {k: "L\t9"})
        m2 = bytearray(stored_member(t2, [30001, 20000]))
        m2[10 + 5 + 30001 + 3] ^= 0x5A
        out[f"stored_nlen_back{back}"] = bytes(m2)
    m = member(gfa(300, {400: "L\tBADKEY\t+\t1\t-\t0M"}).replace(b"BADKEY", b"\xff\xfe"))
    out["trunc_bad_utf8_key"] = m[: int(len(m) * 0.8)]
    m = member(gfa(300))
    full = gzip.decompress(m)
    # truncated inside a line: the partial last line never reaches the parser
    cut = len(m) - 30
    out["trunc_mid_line"] = m[:cut]
    out["multi_member_trunc"] = member(full[: len(full) // 3]) + member(gfa(50, {3: "L\tx"}))[:-12]
    # plain files (name without .gz): the export of the lines before a failing one, rendered from
    # the same input by the native build
    out["plain:malformed_after_edges"] = gfa(200, {700: "L\t1\t+\t2"})
    out["plain:bad_key_then_malformed"] = gfa(200, {300: "L\tBADKEY\t+\t1\t-\t0M", 650: "E\t1"}).replace(
        b"BADKEY", b"\xc3\x28")
    out["plain:unknown_then_malformed"] = gfa(200, {250: "Y\ty", 600: "C\t1\t+"})
    return out


def main() -> None:
    sys.path.insert(0, REF)
    from gfa2network import cli, parse_gfa  # noqa: E402  (the reference)

    INPUTS.mkdir(parents=True, exist_ok=True)
    for f in INPUTS.iterdir():
        f.unlink()
    doc = {}
    for name, blob in inputs().items():
        path = INPUTS / (f"{name[6:]}.gfa" if name.startswith("plain:") else f"{name}.gfa.gz")
        path.write_bytes(blob)
        case = {"file": path.name, "parse": {}, "export": {}}
        for mname, mode in MODES.items():
            for verbose in (False, True):
                err = io.StringIO()
                exc = None
                with warnings.catch_warnings(record=True) as w:
                    warnings.simplefilter("always")
                    try:
                        with contextlib.redirect_stderr(err), contextlib.redirect_stdout(io.StringIO()):
                            parse_gfa(str(path), build_graph=False, build_matrix=True, return_node_list=True,
                                      verbose=verbose, **mode)
                    except Exception as e:  # noqa: BLE001 - recorded as data
                        exc = [type(e).__name__, str(e)]
                case["parse"][f"{mname}|{int(verbose)}"] = {
                    "exc": exc, "stderr": err.getvalue(),
                    "warnings": [str(x.message) for x in w if issubclass(x.category, RuntimeWarning)]}
        with tempfile.TemporaryDirectory() as td:
            for bidir in (False, True):
                dest = Path(td) / "edges.tsv"
                if dest.exists():
                    dest.unlink()
                argv = ["export", str(path), "--format", "edge-list", "--output", str(dest)]
                if bidir:
                    argv.insert(4, "--bidirected")
                exc = None
                with warnings.catch_warnings(record=True) as w:
                    warnings.simplefilter("always")
                    try:
                        cli.main(argv)
                    except Exception as e:  # noqa: BLE001
                        exc = [type(e).__name__, str(e)]
                text = dest.read_bytes() if dest.exists() else b""
                case["export"][str(int(bidir))] = {  # the bytes written: small ones inline, else a digest
                    "text_b64": base64.b64encode(text).decode() if len(text) <= 2048 else None,
                    "text_sha256": hashlib.sha256(text).hexdigest(), "text_len": len(text), "exc": exc,
                    "warnings": [str(x.message) for x in w if issubclass(x.category, RuntimeWarning)]}
        doc[name] = case
        print(name, case["parse"]["default|0"]["exc"], case["parse"]["default|0"]["warnings"])
    (HERE / "expected" / "gzip_prefix.json").write_text(json.dumps(doc, indent=0, sort_keys=True))


if __name__ == "__main__":
    main()
