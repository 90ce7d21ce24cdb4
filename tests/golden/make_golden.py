#!/usr/bin/env python3
"""Generate the golden parity fixtures from the REAL reference (sclipman/gfa2network).

Runs ONLY in the build container, where the pure-Python reference is importable
from /root/reference.  Nothing here is imported by the product,
by the GPU tests at run time, or by bench.py: the committed outputs under
tests/golden/ are plain data (inputs and expected outputs).

What is pinned, per (input, mode, weight_tag, dtype) "combo":
  * `ret`  = what `parse_gfa(path, build_graph=False, build_matrix=True,
             return_node_list=..., **mode)` returns (builders.py:30-299):
             COO in stream order (rows/cols/data, duplicates unsummed) or the
             MAX-SYM CSR (builders.py:282-283), with format, index dtype, data dtype;
  * `csr`  = `convert_format(ret, "csr")` (utils.py:40-63, cli.py:239);
  * node list (builders.py:284-288) as a raw-bytes blob + offsets, and whether the
    str() decode raises;
  * exception type + message (parser.py / builders.py / numpy cast) and the
    RuntimeWarnings emitted (parser.py:117-131), and the verbose stdout/stderr.

Environment recorded in meta.json: python / numpy / scipy versions.
"""
from __future__ import annotations

import contextlib
import gzip
import io
import json
import os
import struct
import sys
import warnings
from pathlib import Path

import numpy as np

REF = "/root/reference"
HERE = Path(__file__).resolve().parent
INPUTS = HERE / "inputs"

MODES = {
    "default": {},
    "undirected": {"directed": False},
    "asym": {"asymmetric": True},
    "undirected_asym": {"directed": False, "asymmetric": True},
    "bidir": {"bidirected": True},
    "bidir_undirected": {"bidirected": True, "directed": False},
    "bidir_keep": {"bidirected": True, "keep_directed_bidir": True},
    "bidir_keep_asym": {"bidirected": True, "keep_directed_bidir": True, "asymmetric": True},
    "keep_only": {"keep_directed_bidir": True},
    "keep_only_undirected": {"keep_directed_bidir": True, "directed": False},
    "strip": {"strip_orientation": True},
    "strip_bidir": {"strip_orientation": True, "bidirected": True},
}
DTYPES = ["bool", "int8", "int32", "float32", "float64"]

# ---------------------------------------------------------------------------
# Small hand-written inputs: SURVEY.md Appendix A.5 known-answer cases.
# ---------------------------------------------------------------------------
T = "\t"


def _l(*f):
    return (T.join(f) + "\n").encode()


SMALL: dict[str, bytes] = {
    # the reference's own sample (tests/test_matrix_asym.py:6)
    "sample": b"S\ts1\t4\nS\ts2\t4\nL\ts1\t+\ts2\t-\t0M\n",
    # tests/test_parser.py:8
    "sample_path": b"S\ts1\tACGT\nS\ts2\tTTTT\nL\ts1\t+\ts2\t-\t0M\nP\tp1\ts1+,s2-\t*\n",
    # weights 5/-3/0/1.5/-7/"x"/9 incl. a duplicate tag, dup edges, reverse edge
    "w": b"".join([
        _l("S", n, "*") for n in "abcdef"
    ] + [
        _l("L", "a", "+", "b", "+", "0M", "RC:i:5"),
        _l("L", "b", "+", "c", "-", "0M", "RC:i:-3"),
        _l("L", "c", "-", "d", "+", "0M", "RC:i:0"),
        _l("L", "d", "+", "e", "+", "0M", "RC:f:1.5"),
        _l("L", "e", "+", "a", "-", "0M", "RC:i:-7"),
        _l("L", "f", "+", "a", "+", "0M", "RC:Z:x"),
        _l("L", "a", "+", "f", "-", "0M", "RC:i:1", "RC:i:9"),
        _l("L", "a", "+", "b", "+", "0M", "RC:i:2"),
        _l("L", "b", "+", "a", "+", "0M", "RC:i:4"),
        _l("L", "c", "+", "c", "+", "0M", "RC:f:-2.25"),
    ]),
    # int8 wrap-around: 100 + 100 -> -56
    "d": b"S\ta\nS\tb\n" + _l("L", "a", "+", "b", "+", "*", "RC:i:100") * 2,
    "crlf": b"S\ta\t*\r\nS\tb\t*\r\nL\ta\t+\tb\t+\t0M\tRC:i:3\r\nL\tb\t-\ta\t+\t0M\r\n",
    "blank_comment": b"S\ta\n\n# comment\nL\ta\t+\tb\t-\t*\nX\tlater\n",
    "gfa2_e_dollar": b"S\ts1\t6\tACGTAC\nS\ts2\t6\tACGTAC\nE\t*\ts1+\ts2-\t0\t6$\t0\t6$\t6M\tRC:i:2\n",
    "gfa2_e_ints": b"E\te1\ts1+\ts2-\t0\t6\t0\t6\t6M\tRC:i:2\nE\te2\ts2-\ts3+\t 1\t+2\t3_0\t4\t*\n",
    "gfa2_e_short": b"E\te1\ts1\t+\ts2\t-\tRC:i:3\n",
    "gfa2_style_l": b"L\ta+\tb-\t0M\tRC:i:4\nL\tc\td\t*\t*\nL\te+-+\tf--\t*\t*\nL\tg-\th\t*\tRC:i:2\tRC:f:2.5\n",
    "short_l": b"S\ta\nL\ta\t+\tb\n",
    "short_p": b"S\ta\nP\tp1\n",
    "short_o": b"S\ta\nO\to1\n",
    "short_s": b"S\ta\nS\n",
    "short_s_eof": b"S\ta\nS",
    "short_e": b"E\te1\ts1\t+\ts2\n",
    "short_c": b"C\ta\t+\tb\n",
    "dup_s": b"S\tb\nS\ta\nS\tb\nL\tc\t+\ta\t+\t*\n",
    "containment": b"S\ta\nS\tb\nC\ta\t+\tb\t-\t10\t5M\tRC:i:6\nC\tx\ty+\t1\t2\tz-\t3\t4\t*\tRC:i:7\n",
    "weird_tags": b"".join([
        _l("L", "a", "+", "b", "+", "*", "RC:i:1_0"),
        _l("L", "b", "+", "c", "+", "*", "RC:f:1e400"),
        _l("L", "c", "+", "d", "+", "*", "RC:f:nan"),
        _l("L", "d", "+", "e", "+", "*", "RC:i: 7 "),
        _l("L", "e", "+", "f", "+", "*", "RC:f:-nan"),
        _l("L", "f", "+", "g", "+", "*", "RC:f:1_0.2_5e-1"),
        _l("L", "g", "+", "h", "+", "*", "RC:i:5", "RC:Z:x"),
        _l("L", "h", "+", "i", "+", "*", "RC:i:5", "RC:i:bad"),
        _l("L", "i", "+", "j", "+", "*", "RC:B:1,2"),
        _l("L", "j", "+", "k", "+", "*", "RC:f:-inFinity"),
        _l("L", "k", "+", "l", "+", "*", "RC:f:.5"),
        _l("L", "l", "+", "m", "+", "*", "RC:f:5."),
        _l("L", "m", "+", "n", "+", "*", "RC:f:0.1"),
        _l("L", "n", "+", "o", "+", "*", "RC::1"),
        _l("L", "o", "+", "p", "+", "*", "RC:i:+0012"),
        _l("L", "p", "+", "q", "+", "*", "RC:i:1__0"),
        _l("L", "q", "+", "r", "+", "*", "RC:f:1e-400"),
        _l("L", "r", "+", "s", "+", "*", "RC:f:-0.0"),
        _l("L", "s", "+", "t", "+", "*", "rc:i:3"),
        _l("L", "t", "+", "u", "+", "*", "RC:i:3:4"),
        "L\tu\t+\tv\t+\t*\tRC:i:\u0663\u0664\n".encode(),
        "L\tv\t+\tw\t+\t*\tRC:f:\u00a01.25\u3000\n".encode(),
        b"L\tw\t+\tx\t+\t*\tRC:i:\xff5\n",
        _l("L", "x", "+", "y", "+", "*", "RC:f:123456789012345678901234567890e-20"),
        _l("L", "y", "+", "z", "+", "*", "RC:f:2.2250738585072011e-308"),
        _l("L", "z", "+", "A", "+", "*", "RC:i:9007199254740993"),
        _l("L", "A", "+", "B", "+", "*", "RC:i:-0"),
        _l("L", "B", "+", "C", "+", "*", "RC:i:" + "1" * 4301),
        _l("L", "C", "+", "D", "+", "*", "RC:i:" + "1" * 300),
        _l("L", "D", "+", "E", "+", "*", "RC:f:" + "1" * 400 + "e-390"),
        _l("L", "E", "+", "F", "+", "*", "RC:f:0." + "0" * 500 + "1e500"),
        _l("L", "F", "+", "G", "+", "*", "RC:f:4.9406564584124654e-324"),
        _l("L", "G", "+", "H", "+", "*", "RC:f:1e", "RC:f:e5"),
        _l("L", "H", "+", "I", "+", "*", "RC:f:_1", "RC:i:1_"),
        _l("L", "I", "+", "J", "+", "*", "RC:f:InF", "RC:f:nAn"),
        _l("L", "J", "+", "K", "+", "*", "RC:f:+.e1"),
        _l("L", "K", "+", "L", "+", "*", "RC:f:1.7976931348623158e308"),
        _l("L", "L", "+", "M", "+", "*", "RC:f:1.7976931348623159e308"),
        "L\tM\t+\tN\t+\t*\tRC:f:\uff11\uff12.5\n".encode(),
        b"L\tN\t+\tO\t+\t*\tRC:i:1\x00\n",
        b"L\tO\t+\tP\t+\t*\tRC:i:\x0b12\x0c\r\n",
    ]),
    "sx": b"S\ta\nSx\tfoo\nLL\ta\t+\tb\t+\nL\ta\t+\tb\t+\t*\n",
    "strip_names": _l("L", "a+", "+", "b-", "-", "*") + _l("L", "a", "-", "b", "+", "*"),
    "self_loop": _l("S", "a") + _l("L", "a", "+", "a", "+", "*") + _l("L", "a", "+", "a", "-", "*"),
    "trailing_tab": b"S\ta\nL\ta\t+\tb\t+\t*\t\nL\tb\t+\tc\t+\t*\tRC:i:2\t\n",
    "empty_name": b"S\t\nL\t\t+\tb\t+\t*\nL\tb\t+\t\t-\t*\n",
    "no_trailing_newline": b"S\ta\nS\tb\nL\ta\t+\tb\t-\t*",
    "nan_both_sides": _l("L", "a", "+", "b", "+", "*", "RC:f:nan") + _l("L", "b", "+", "a", "+", "*", "RC:i:1"),
    "neg_weights": _l("L", "a", "+", "b", "+", "*", "RC:i:-1") + _l("L", "b", "+", "c", "+", "*", "RC:i:-2")
    + _l("L", "c", "+", "b", "+", "*", "RC:i:5") + _l("L", "c", "+", "d", "+", "*", "RC:i:0"),
    "nonascii_first": b"S\ta\n\xffjunk\nL\ta\t+\tb\t+\t*\n",
    "nonascii_second_unknown": b"S\ta\n#c\n\xffjunk\nL\ta\t+\tb\t+\t*\n",
    "warn_then_error": b"S\ta\nW\tw\nL\ta\t+\n",
    "error_then_warn": b"S\ta\nL\ta\t+\nW\tw\n",
    "h_f_silent": b"H\tVN:Z:1.0\nF\tx\nS\ta\n",
    "bad_utf8_ori": b"S\ta\nL\ta\t+\tb\t\xff\t*\n",
    "bad_utf8_ori_e": b"E\te\ta\t\xfe\tb\t+\n",
    "bad_utf8_name": b"S\t\xff\xfe\nS\tok\nL\tok\t+\t\xff\xfe\t+\t*\n",
    "utf8_names": "S\t\u00e9t\u00e9\nL\t\u00e9t\u00e9\t+\t\u65e5\u672c\t-\t*\n".encode(),
    "weird_ori": _l("L", "a", "+", "b", "x", "*") + _l("L", "a", "-", "b", "", "*") + _l("L", "b", "+", "a", "+:x", "*")
    + _l("S", "a:+"),
    "huge_int_weight": _l("S", "a") + _l("L", "a", "+", "b", "+", "*", "RC:i:" + "9" * 400),
    "overflow_int8": _l("L", "a", "+", "b", "+", "*", "RC:i:300") + _l("L", "a", "+", "c", "+", "*", "RC:f:nan"),
    "nan_first_int": _l("L", "a", "+", "c", "+", "*", "RC:f:nan") + _l("L", "a", "+", "b", "+", "*", "RC:i:300"),
    "inf_weight": _l("L", "a", "+", "b", "+", "*", "RC:f:inf") + _l("L", "b", "+", "c", "+", "*", "RC:f:-inf"),
    "empty_file": b"",
    "only_header": b"H\tVN:Z:1.0\n",
    "only_segments": b"S\ta\nS\tb\n",
    "blank_lines_only": b"\n\n\n",
    "p_o_records": b"S\ta\nP\tp\ta+,b-\t*\nO\to\ta+ b-\nL\ta\t+\tb\t+\t*\n",
    "l_gfa1_empty_u_gfa2": b"L\t\tb\t*\t*\n",
    "many_tabs": b"L\ta\t+\tb\t+\t\t\t\t\tRC:i:4\n",
    "cr_only_line": b"S\ta\n\r\nL\ta\t+\tb\t+\t*\n",
}


def _float_dup_row() -> bytes:
    """>=3 float duplicates in rows of >16 entries (SciPy std::sort order, A.3)."""
    rng = np.random.default_rng(7)
    out = []
    vals = [1e16, 1.0, -1e16, 0.1, 3.3, -2.7, 1e-3, 7.0]
    for r in range(3):
        for k in range(40):
            c = int(rng.integers(0, 12))
            v = vals[int(rng.integers(0, len(vals)))] * (1 + int(rng.integers(0, 3)))
            out.append(_l("L", f"r{r}", "+", f"c{c}", "+", "*", f"RC:f:{v!r}"))
    # the transposed direction too (MAX-SYM reads both A and A.T orders)
    for k in range(40):
        c = int(rng.integers(0, 12))
        v = vals[int(rng.integers(0, len(vals)))]
        out.append(_l("L", f"c{c}", "+", "r0", "+", "*", f"RC:f:{v!r}"))
    return b"".join(out)


SMALL["float_dups_long_rows"] = _float_dup_row()


def synthetic_small(n_s: int, n_l: int, seed: int, rc: bool) -> bytes:
    """Synthetic pangenome-like GFA in the SURVEY §8(d) shape (small, numpy PCG64)."""
    rng = np.random.default_rng(seed)
    lines = ["H\tVN:Z:1.0\n"]
    seqlen = rng.geometric(1.0 / 8.0, size=n_s)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    for i in range(n_s):
        seq = acgt[rng.integers(0, 4, size=int(seqlen[i]))].tobytes().decode()
        lines.append(f"S\t{i + 1}\t{seq}\n")
    src = rng.integers(1, n_s + 1, size=n_l)
    dst = np.minimum(src + rng.geometric(0.3, size=n_l), n_s)
    o1 = np.where(rng.random(n_l) < 0.9, "+", "-")
    o2 = np.where(rng.random(n_l) < 0.9, "+", "-")
    k = rng.integers(1, 100, size=n_l)
    for j in range(n_l):
        tag = f"\tRC:i:{k[j]}" if rc else ""
        lines.append(f"L\t{src[j]}\t{o1[j]}\t{dst[j]}\t{o2[j]}\t0M{tag}\n")
    return "".join(lines).encode()


def _bits_hex(a: np.ndarray) -> str:
    return np.ascontiguousarray(a).tobytes().hex()


def _exc(e: BaseException) -> dict:
    return {"type": type(e).__name__, "msg": str(e)}


def run_combo(gfa2network, path: str, mode: dict, weight_tag, dtype: str, arrays: dict, key: str):
    """Run the reference for one combo; store arrays under `key/` and return meta."""
    from gfa2network import parse_gfa, convert_format
    import scipy.sparse as sp

    meta: dict = {"mode": mode, "weight_tag": weight_tag, "dtype": dtype}
    kw = dict(build_graph=False, build_matrix=True, weight_tag=weight_tag, dtype=dtype, **mode)

    def call(**extra):
        out_buf, err_buf = io.StringIO(), io.StringIO()
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            exc = None
            res = None
            try:
                with contextlib.redirect_stdout(out_buf), contextlib.redirect_stderr(err_buf):
                    res = parse_gfa(path, **kw, **extra)
            except Exception as e:  # noqa: BLE001 - we record the reference's exception
                exc = e
        warns = [{"category": x.category.__name__, "msg": str(x.message)} for x in w]
        return res, exc, warns, out_buf.getvalue(), err_buf.getvalue()

    # 1) return_node_list=True, raw_bytes_id=True: matrix + exact node bytes
    res, exc, warns, so, se = call(return_node_list=True, raw_bytes_id=True)
    meta["warnings"] = warns
    if exc is not None:
        meta["exception"] = _exc(exc)
        return meta
    A, nodes = res
    blob = b"".join(nodes)
    offs = np.zeros(len(nodes) + 1, dtype=np.int64)
    if nodes:
        offs[1:] = np.cumsum([len(x) for x in nodes])
    arrays[f"{key}/names_blob"] = np.frombuffer(blob, dtype=np.uint8).copy()
    arrays[f"{key}/names_offsets"] = offs
    meta["n"] = int(A.shape[0])
    meta["shape"] = list(A.shape)

    def dump(M, pre):
        d = {"format": M.format, "dtype": str(M.dtype), "nnz": int(M.nnz)}
        if M.format == "coo":
            d["index_dtype"] = str(M.row.dtype)
            d["has_canonical_format"] = bool(M.has_canonical_format)
            arrays[f"{key}/{pre}/row"] = np.asarray(M.row)
            arrays[f"{key}/{pre}/col"] = np.asarray(M.col)
        else:
            d["index_dtype"] = str(M.indices.dtype)
            d["indptr_dtype"] = str(M.indptr.dtype)
            d["has_canonical_format"] = bool(M.has_canonical_format)
            arrays[f"{key}/{pre}/indptr"] = np.asarray(M.indptr)
            arrays[f"{key}/{pre}/indices"] = np.asarray(M.indices)
        arrays[f"{key}/{pre}/data"] = np.asarray(M.data)
        return d

    meta["ret"] = dump(A, "ret")
    C = convert_format(A, "csr")
    meta["csr"] = dump(C, "csr")
    # 2) str node list: does node.decode() raise? (builders.py:287)
    res2, exc2, _, _, _ = call(return_node_list=True)
    meta["node_decode_exception"] = _exc(exc2) if exc2 is not None else None
    # 3) verbose strings (builders.py:257-261)
    _, _, _, so3, se3 = call(return_node_list=False, verbose=True)
    meta["verbose_stdout"] = so3
    meta["verbose_stderr"] = se3
    return meta


def main() -> None:
    sys.path.insert(0, REF)
    import gfa2network  # noqa: F401  (the reference, container-only)
    import hashlib
    import scipy

    INPUTS.mkdir(parents=True, exist_ok=True)
    files: dict[str, Path] = {}
    for name, data in SMALL.items():
        p = INPUTS / f"{name}.gfa"
        p.write_bytes(data)
        files[name] = p
    # gzip inputs: multi-member, and a BGZF-style FEXTRA member
    w = SMALL["w"]
    half = len(w) // 2
    cut = w.rfind(b"\n", 0, half) + 1
    (INPUTS / "w_multimember.gfa.gz").write_bytes(gzip.compress(w[:cut], mtime=0) + gzip.compress(w[cut:], mtime=0))
    files["w_multimember_gz"] = INPUTS / "w_multimember.gfa.gz"
    (INPUTS / "w_bgzf.gfa.gz").write_bytes(bgzf_like(w))
    files["w_bgzf_gz"] = INPUTS / "w_bgzf.gfa.gz"
    syn = synthetic_small(3000, 12000, seed=1, rc=True)
    (INPUTS / "syn3k.gfa.gz").write_bytes(gzip.compress(syn, mtime=0))
    files["syn3k_gz"] = INPUTS / "syn3k.gfa.gz"
    files["drb1"] = INPUTS / "DRB1-3123_unsorted.gfa"

    env = {"python": sys.version.split()[0], "numpy": np.__version__, "scipy": scipy.__version__,
           "reference": "sclipman/gfa2network 1.0 @ 2025-07-04"}
    pool: dict[str, np.ndarray] = {}
    doc = {"env": env, "inputs": {}}
    big = {"drb1", "syn3k_gz"}
    for name, path in files.items():
        arrays: dict[str, np.ndarray] = {}
        metas = {}
        raw = gzip.decompress(path.read_bytes()) if str(path).endswith(".gz") else path.read_bytes()
        has_rc = b"RC:" in raw
        for mname, mode in MODES.items():
            for wt in ([None, "RC"] if has_rc else [None]):
                for dt in DTYPES:
                    if name in big and (dt not in ("float64", "bool", "int8")
                                        or mname in ("strip", "keep_only_undirected", "bidir_undirected")):
                        continue
                    key = f"{mname}|{wt or '-'}|{dt}"
                    meta = run_combo(None, str(path), mode, wt, dt, arrays, key)
                    # content-addressed array pool: identical arrays stored once
                    refs = {}
                    for k in [k for k in arrays if k.startswith(key + "/")]:
                        a = arrays.pop(k)
                        h = hashlib.sha256(a.dtype.str.encode() + a.tobytes()).hexdigest()[:20]
                        pool.setdefault(h, a)
                        refs[k[len(key) + 1:]] = h
                    meta["arrays"] = refs
                    metas[key] = meta
        doc["inputs"][name] = {"file": path.name, "combos": metas}
        print(f"{name}: {len(metas)} combos; pool now {len(pool)} arrays")
    outdir = HERE / "expected"
    outdir.mkdir(exist_ok=True)
    for f in outdir.iterdir():
        f.unlink()
    (outdir / "golden.json").write_text(json.dumps(doc, sort_keys=True, separators=(",", ":")))
    np.savez_compressed(outdir / "pool.npz", **pool)


def bgzf_like(data: bytes, block: int = 64) -> bytes:
    """Concatenated gzip members, each with an FEXTRA 'BC' subfield holding BSIZE-1
    (the BGZF layout of htslib's bgzip; blocks here are tiny on purpose)."""
    import zlib

    out = bytearray()
    for i in range(0, len(data), block):
        chunk = data[i:i + block]
        co = zlib.compressobj(6, zlib.DEFLATED, -15)
        cdata = co.compress(chunk) + co.flush()
        xlen = 6
        total = 10 + 2 + xlen + len(cdata) + 8  # header + XLEN + extra + cdata + trailer
        hdr = bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF]) + struct.pack("<H", xlen)
        hdr += b"BC" + struct.pack("<HH", 2, total - 1)
        out += hdr + cdata + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk) & 0xFFFFFFFF)
    # BGZF EOF marker block (empty member)
    out += bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    return bytes(out)


if __name__ == "__main__":
    os.chdir(HERE)
    main()
