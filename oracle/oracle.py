"""ctypes wrapper of the CPU restatement (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY — the checker.  Imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg; never by the gfa2network_amd product.

`run(data, **mode)` returns an `OracleResult` with everything the reference computes for
one input: stream-order COO, the SUM CSR (convert_format "csr") and, when the mode is
MAX-SYM, the A.maximum(A.T) CSR; `to_raw(...)` re-expresses it as the product's
`RawResult` so the same host-side finalize() turns both into scipy objects.
"""
from __future__ import annotations

import ctypes
import subprocess
from dataclasses import dataclass
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "liboracle.so"
DTYPES = {"bool": 0, "int8": 1, "int32": 2, "float32": 3, "float64": 4}


class _Opts(ctypes.Structure):
    _fields_ = [
        ("directed", ctypes.c_int32), ("bidirected", ctypes.c_int32), ("keep_directed_bidir", ctypes.c_int32),
        ("asymmetric", ctypes.c_int32), ("strip_orientation", ctypes.c_int32), ("dtype", ctypes.c_int32),
        ("weight_tag", ctypes.c_char_p),
    ]


class _Res(ctypes.Structure):
    _fields_ = [
        ("status", ctypes.c_int32), ("err_line", ctypes.c_int64), ("err_index", ctypes.c_int64),
        ("err_value", ctypes.c_double), ("err_detail", ctypes.c_void_p), ("err_detail_len", ctypes.c_int64),
        ("has_warning", ctypes.c_int32), ("warn_byte", ctypes.c_int32), ("warn_line", ctypes.c_int64),
        ("n_lines", ctypes.c_int64), ("n_records", ctypes.c_int64), ("n_records_before_error", ctypes.c_int64),
        ("n_nodes", ctypes.c_int64), ("names_blob", ctypes.c_void_p), ("names_offsets", ctypes.c_void_p),
        ("n_trip", ctypes.c_int64), ("rows", ctypes.c_void_p), ("cols", ctypes.c_void_p),
        ("weights", ctypes.c_void_p), ("data_cast", ctypes.c_void_p),
        ("sum_nnz", ctypes.c_int64), ("sum_indptr", ctypes.c_void_p), ("sum_indices", ctypes.c_void_p),
        ("sum_data", ctypes.c_void_p),
        ("has_maxsym", ctypes.c_int32), ("ms_nnz", ctypes.c_int64), ("ms_indptr", ctypes.c_void_p),
        ("ms_indices", ctypes.c_void_p), ("ms_data", ctypes.c_void_p), ("sum_sorted_input", ctypes.c_int32),
        ("n_cast_overflow", ctypes.c_int64),
    ]


_lib = None


def build() -> Path:
    """Compile the restatement (make -C oracle)."""
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        lib = ctypes.CDLL(str(LIB))
        lib.oracle_build.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(_Opts),
                                     ctypes.POINTER(ctypes.POINTER(_Res))]
        lib.oracle_build.restype = ctypes.c_int
        lib.oracle_free.argtypes = [ctypes.POINTER(_Res)]
        lib.oracle_free.restype = None
        _lib = lib
    return _lib


def _arr(addr, count, dtype):
    dtype = np.dtype(dtype)
    if not addr or count == 0:
        return np.zeros(0, dtype=dtype)
    return np.frombuffer((ctypes.c_char * (count * dtype.itemsize)).from_address(addr), dtype=dtype).copy() if count else np.empty(0, dtype)


@dataclass
class OracleResult:
    status: int
    err_line: int
    err_index: int
    err_value: float
    err_detail: bytes
    has_warning: bool
    warn_byte: int
    warn_line: int
    n_lines: int
    n_records: int
    n_records_before_error: int
    n_nodes: int
    names_blob: np.ndarray
    names_offsets: np.ndarray
    dtype: np.dtype
    rows: np.ndarray | None = None
    cols: np.ndarray | None = None
    weights: np.ndarray | None = None
    data: np.ndarray | None = None
    sum_indptr: np.ndarray | None = None
    sum_indices: np.ndarray | None = None
    sum_data: np.ndarray | None = None
    maxsym: bool = False
    ms_indptr: np.ndarray | None = None
    ms_indices: np.ndarray | None = None
    ms_data: np.ndarray | None = None
    sum_sorted_input: bool = True
    n_cast_overflow: int = 0


def run(data: bytes, *, directed=True, bidirected=False, keep_directed_bidir=False, asymmetric=False,
        strip_orientation=False, dtype="float64", weight_tag=None) -> OracleResult:
    lib = load()
    o = _Opts(int(directed), int(bidirected), int(keep_directed_bidir), int(asymmetric), int(strip_orientation),
              DTYPES[np.dtype(dtype).name], weight_tag.encode() if weight_tag else None)
    buf = np.frombuffer(bytes(data), dtype=np.uint8)
    res = ctypes.POINTER(_Res)()
    lib.oracle_build(buf.ctypes.data if buf.size else None, buf.size, ctypes.byref(o), ctypes.byref(res))
    r = res.contents
    dt = np.dtype(dtype)
    try:
        offs = _arr(r.names_offsets, r.n_nodes + 1, np.int64)
        out = OracleResult(
            status=r.status, err_line=r.err_line, err_index=r.err_index, err_value=r.err_value,
            err_detail=ctypes.string_at(r.err_detail, r.err_detail_len) if r.err_detail else b"",
            has_warning=bool(r.has_warning), warn_byte=r.warn_byte, warn_line=r.warn_line,
            n_lines=r.n_lines, n_records=r.n_records, n_records_before_error=r.n_records_before_error,
            n_nodes=r.n_nodes, names_blob=_arr(r.names_blob, int(offs[-1]) if len(offs) else 0, np.uint8),
            names_offsets=offs, dtype=dt)
        if r.status == 0:
            out.rows = _arr(r.rows, r.n_trip, np.int64)
            out.cols = _arr(r.cols, r.n_trip, np.int64)
            out.weights = _arr(r.weights, r.n_trip, np.float64)
            out.data = _arr(r.data_cast, r.n_trip, dt)
            out.sum_indptr = _arr(r.sum_indptr, r.n_nodes + 1, np.int64)
            out.sum_indices = _arr(r.sum_indices, r.sum_nnz, np.int64)
            out.sum_data = _arr(r.sum_data, r.sum_nnz, dt)
            out.sum_sorted_input = bool(r.sum_sorted_input)
            out.n_cast_overflow = int(r.n_cast_overflow)
            if r.has_maxsym:
                out.maxsym = True
                out.ms_indptr = _arr(r.ms_indptr, r.n_nodes + 1, np.int64)
                out.ms_indices = _arr(r.ms_indices, r.ms_nnz, np.int64)
                out.ms_data = _arr(r.ms_data, r.ms_nnz, dt)
        elif r.status in (10, 11, 12):
            out.n_nodes = r.n_nodes
    finally:
        lib.oracle_free(res)
    return out


def to_raw(o: OracleResult, output: str = "parse"):
    """The oracle's answer as the product's RawResult (output "parse" or "csr")."""
    from gfa2network_amd._native import RawResult  # host-side dataclass only (no GPU)

    raw = RawResult(status=o.status, err_line=o.err_line, err_index=o.err_index, err_value=o.err_value,
                    err_detail=o.err_detail, has_warning=o.has_warning, warn_byte=o.warn_byte,
                    warn_line=o.warn_line, n_lines=o.n_lines, n_records=o.n_records,
                    n_records_before_error=o.n_records_before_error, n_nodes=o.n_nodes,
                    names_blob=o.names_blob, names_offsets=o.names_offsets, dtype=o.dtype,
                    n_cast_overflow=o.n_cast_overflow)
    if o.status != 0:
        return raw
    if o.maxsym:
        raw.format = "csr"
        raw.indptr = o.ms_indptr.astype(np.int32)
        raw.indices = o.ms_indices.astype(np.int32)
        raw.data = o.ms_data
    elif output == "parse":
        raw.format = "coo"
        raw.rows = o.rows.astype(np.int32)
        raw.cols = o.cols.astype(np.int32)
        raw.data = o.data
    else:
        raw.format = "csr"
        raw.indptr = o.sum_indptr.astype(np.int32)
        raw.indices = o.sum_indices.astype(np.int32)
        raw.data = o.sum_data
    return raw


def export_edge_list(data: bytes, *, bidirected: bool = False):
    """CPU restatement of ``export --format edge-list`` (cli.py:264-281) for the tests.

    The reference's loop writes ``f"{u.decode()}\\t{v.decode()}\\n"`` for every L/E/C record the
    parser yields; u / v are the record keys that the directed, keep-orientation matrix build
    mints for the same record (builders.py:199-228, bidirected ``u:ori``), so the lines are
    the stream-order COO's row / col names.  Returns ``(text, error, first)``: error = None or
    ``(kind, payload)``: ("status", the failing OracleResult) for a parse failure (text = the
    lines before the failing line), ("decode", key bytes) for a key that is not UTF-8; first =
    the full-input OracleResult (its warning flags).
    """
    o = run(data, directed=True, bidirected=bidirected, keep_directed_bidir=True, asymmetric=True, dtype="bool")
    err = None
    first = o
    if o.status != 0:
        if o.err_line < 0:
            return b"", ("status", o), first
        err = ("status", o)
        arr = np.frombuffer(bytes(data), dtype=np.uint8)
        nl = np.flatnonzero(arr == 0x0A)
        end = 0 if o.err_line == 0 else int(nl[o.err_line - 1]) + 1
        o = run(arr[:end].tobytes(), directed=True, bidirected=bidirected, keep_directed_bidir=True,
                asymmetric=True, dtype="bool")
        assert o.status == 0, "the prefix before a failing line parses"
    blob, offs = o.names_blob.tobytes(), o.names_offsets
    names = [blob[offs[i]:offs[i + 1]] for i in range(o.n_nodes)]
    out = []
    for r, c in zip(o.rows.tolist(), o.cols.tolist()):
        for k in (r, c):
            try:
                names[k].decode()
            except UnicodeDecodeError:
                return b"".join(out), ("decode", names[k]), first
        out.append(names[r] + b"\t" + names[c] + b"\n")
    return b"".join(out), err, first
