"""Loading and comparing the golden fixtures made by tests/golden/make_golden.py.

A "combo" is (input, mode, weight_tag, dtype).  `outcome(...)` runs one combo through any
engine that returns the product's RawResult (the GPU library, or the oracle re-expressed
as a RawResult) plus the shared host-side finalize(), and `check(...)` compares it with
what the reference produced: exception type/message, RuntimeWarnings, verbose output,
returned format/dtype/index dtype/arrays (bit for bit), convert_format(..., "csr"), and
the node list.
"""
from __future__ import annotations

import contextlib
import gzip
import io
import json
import warnings
from functools import lru_cache
from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden"


@lru_cache(maxsize=1)
def doc():
    return json.loads((GOLDEN / "expected" / "golden.json").read_text())


@lru_cache(maxsize=1)
def pool():
    with np.load(GOLDEN / "expected" / "pool.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def input_path(name: str) -> Path:
    return GOLDEN / "inputs" / doc()["inputs"][name]["file"]


def input_bytes(name: str) -> bytes:
    p = input_path(name)
    raw = p.read_bytes()
    return gzip.decompress(raw) if p.name.endswith(".gz") else raw


def combos(names=None):
    d = doc()["inputs"]
    for name in sorted(d) if names is None else names:
        for key in sorted(d[name]["combos"]):
            yield name, key


def combo(name: str, key: str) -> dict:
    return doc()["inputs"][name]["combos"][key]


def arr(ref: str) -> np.ndarray:
    return pool()[ref]


def bits_equal(a: np.ndarray, b: np.ndarray) -> bool:
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.dtype == b.dtype and a.shape == b.shape and a.tobytes() == b.tobytes()


def run_python(fn, *args, **kw):
    """Call fn capturing (result, exception, warnings, stdout, stderr)."""
    out, err = io.StringIO(), io.StringIO()
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        res, exc = None, None
        try:
            with contextlib.redirect_stdout(out), contextlib.redirect_stderr(err):
                res = fn(*args, **kw)
        except Exception as e:  # noqa: BLE001 - the reference's exceptions are part of parity
            exc = e
    warns = [{"category": x.category.__name__, "msg": str(x.message)} for x in w]
    return res, exc, warns, out.getvalue(), err.getvalue()


def check_matrix(M, want: dict, arrays: dict, pre: str) -> list[str]:
    errs = []
    if M.format != want["format"]:
        return [f"{pre}: format {M.format} != {want['format']}"]
    if str(M.dtype) != want["dtype"]:
        errs.append(f"{pre}: dtype {M.dtype} != {want['dtype']}")
    if M.nnz != want["nnz"]:
        errs.append(f"{pre}: nnz {M.nnz} != {want['nnz']}")
    if M.format == "coo":
        if str(M.row.dtype) != want["index_dtype"]:
            errs.append(f"{pre}: index dtype {M.row.dtype} != {want['index_dtype']}")
        for k, v in (("row", M.row), ("col", M.col), ("data", M.data)):
            if not bits_equal(np.asarray(v), arr(arrays[f"{pre}/{k}"])):
                errs.append(f"{pre}/{k} differs")
    else:
        if str(M.indices.dtype) != want["index_dtype"] or str(M.indptr.dtype) != want["indptr_dtype"]:
            errs.append(f"{pre}: index dtypes {M.indices.dtype}/{M.indptr.dtype}")
        for k, v in (("indptr", M.indptr), ("indices", M.indices), ("data", M.data)):
            if not bits_equal(np.asarray(v), arr(arrays[f"{pre}/{k}"])):
                errs.append(f"{pre}/{k} differs")
        if bool(M.has_canonical_format) != want["has_canonical_format"]:
            errs.append(f"{pre}: has_canonical_format {M.has_canonical_format}")
    return errs


def check(name: str, key: str, run_engine, convert) -> list[str]:
    """run_engine(return_node_list, raw_bytes_id, verbose) -> the engine's parse_gfa result
    (or raises); convert(A) -> convert_format(A, "csr").  Returns a list of mismatches."""
    g = combo(name, key)
    errs: list[str] = []
    res, exc, warns, _, _ = run_python(run_engine, True, True, False)
    if warns != g["warnings"]:
        errs.append(f"warnings {warns} != {g['warnings']}")
    if "exception" in g:
        want = g["exception"]
        if exc is None:
            errs.append(f"expected {want['type']}: {want['msg']}, got a result")
        elif type(exc).__name__ != want["type"] or str(exc) != want["msg"]:
            errs.append(f"exception {type(exc).__name__}: {exc} != {want['type']}: {want['msg']}")
        return errs
    if exc is not None:
        return errs + [f"unexpected {type(exc).__name__}: {exc}"]
    A, nodes = res
    a = g["arrays"]
    if list(A.shape) != g["shape"]:
        errs.append(f"shape {A.shape} != {g['shape']}")
    errs += check_matrix(A, g["ret"], a, "ret")
    C = convert(A)
    errs += check_matrix(C, g["csr"], a, "csr")
    blob = b"".join(nodes)
    offs = np.zeros(len(nodes) + 1, dtype=np.int64)
    if nodes:
        offs[1:] = np.cumsum([len(x) for x in nodes])
    if not bits_equal(np.frombuffer(blob, dtype=np.uint8), arr(a["names_blob"])) or not bits_equal(
            offs, arr(a["names_offsets"])):
        errs.append("node list (raw bytes) differs")
    res2, exc2, _, _, _ = run_python(run_engine, True, False, False)
    want2 = g["node_decode_exception"]
    if want2 is None and exc2 is not None:
        errs.append(f"str node list raised {type(exc2).__name__}: {exc2}")
    if want2 is not None and (exc2 is None or type(exc2).__name__ != want2["type"] or str(exc2) != want2["msg"]):
        errs.append(f"str node list: {exc2!r} != {want2}")
    if want2 is None and exc2 is None and res2[1] != [x.decode() for x in nodes]:
        errs.append("str node list differs")
    _, _, _, so, se = run_python(run_engine, False, False, True)
    if so != g["verbose_stdout"] or se != g["verbose_stderr"]:
        errs.append(f"verbose output {so!r}/{se!r} != {g['verbose_stdout']!r}/{g['verbose_stderr']!r}")
    return errs
