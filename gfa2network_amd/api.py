"""parse_gfa / convert_format with the reference's call surface, backed by libg2n.so.

Mirrors the matrix subset of sclipman/gfa2network:
  * ``parse_gfa(path, *, build_graph, build_matrix, ...)``   gfa2network/builders.py:30-299
  * ``convert_format(A, fmt, *, verbose=False)``             gfa2network/utils.py:40-63

Same keyword names, defaults, returned objects (scipy ``coo_matrix`` in stream order, or
the MAX-SYM ``csr_matrix``; node list of ``str`` or raw ``bytes``), exception types and
messages, the one-shot ``RuntimeWarning`` and the ``verbose`` progress strings.  Every
numeric step runs on the GPU; only the Python objects are assembled here.  Graph-object
outputs (NetworkX / igraph, and ``split_on_alignment`` with ``build_graph=True``) are outside
this path's scope and raise ``NotImplementedError``; ``split_on_alignment`` matrix outputs are
served (``_parse_gfa_split``).
"""
from __future__ import annotations

import gzip
import io
import os
import sys
import time
import warnings
import zlib
from pathlib import Path
from typing import Any

import numpy as np
import scipy.sparse as sp

from . import _native as nat
from ._native import RawResult

try:  # the reference's verbose progress draws a tqdm bar when tqdm is importable (utils.py:8-14)
    from tqdm.auto import tqdm

    _HAS_TQDM = True
except Exception:  # noqa: BLE001 - the same broad guard as the reference
    tqdm = None  # type: ignore
    _HAS_TQDM = False

__all__ = ["parse_gfa", "parse_gfa_names", "parse_gfa_sharded", "convert_format", "finalize", "raise_for_status",
           "save_npz"]

# Auto-sharding (BASELINE north_star: byte-range-shard "only when it exceeds one GPU's HBM"): a
# build's device working set is at most about this many bytes per input byte (the lean decimal-id
# MAX-SYM build of C4 peaks near 3x; hash-dictionary, bidirected and weighted builds need more).
WORKING_SET_PER_INPUT_BYTE = 8

_MALFORMED = {
    nat.E_MALFORMED_L: "L", nat.E_MALFORMED_E: "E", nat.E_MALFORMED_C: "C",
    nat.E_MALFORMED_P: "P", nat.E_MALFORMED_O: "O",
}


def raise_for_status(raw: RawResult, dtype: np.dtype, path: Any = None) -> None:
    """Raise exactly what the reference raises for this failure (type and message)."""
    s = raw.status
    if s == nat.OK:
        return
    if s in _MALFORMED:  # parser.py:209, 252, 300, 232, 346
        raise ValueError(f"Malformed {_MALFORMED[s]} record")
    if s == nat.E_INDEX_LIST:  # parser.py:163 fields[1]
        raise IndexError("list index out of range")
    if s == nat.E_INDEX_BYTES:  # parser.py:220-221 u_field[-1] on b""
        raise IndexError("index out of range")
    if s == nat.E_UNICODE:  # the same bytes.decode() the reference calls
        bytes(raw.err_detail).decode()
        raise AssertionError("decode of the reported bytes unexpectedly succeeded")
    if s == nat.E_INT_TOO_LARGE:  # builders.py:209 float(int)
        raise OverflowError("int too large to convert to float")
    if s == nat.E_CAST_OVERFLOW:  # numpy cast in coo_matrix(..., dtype) (builders.py:281)
        raise OverflowError(f"Python integer {int(raw.err_value)} out of bounds for {dtype}")
    if s == nat.E_CAST_INF:
        raise OverflowError("cannot convert float infinity to integer")
    if s == nat.E_CAST_NAN:
        raise ValueError("cannot convert float NaN to integer")
    if s == nat.E_IO:
        err = int(raw.err_index)
        raise OSError(err, os.strerror(err), str(path))
    if s == nat.E_GZIP:  # gzip.open(...) failures (parser.py:108-109)
        sub = int(raw.err_index)
        if sub == 2:
            raise EOFError(raw.message)
        if sub == 3:
            raise zlib.error(raw.message)
        raise gzip.BadGzipFile(raw.message)
    raise RuntimeError(f"{nat.status_name(s)}: {raw.message}")


def _node_list(raw: RawResult, raw_bytes_id: bool) -> list:
    """node_list[idx] = node (raw_bytes_id) or node.decode()  (builders.py:284-288)."""
    offs = raw.names_offsets
    n = 0 if offs is None else len(offs) - 1
    if n == 0:
        return []
    blob = raw.names_blob
    # names never contain b"\n" (lines are split on it): join with "\n" and split once
    jb = nat.join_names(blob, offs)
    if raw_bytes_id:
        return bytes(jb).split(b"\n")
    try:
        return jb.decode().split("\n")
    except UnicodeDecodeError:
        pass
    for i in range(n):  # the first undecodable name in id order raises, as in the reference
        bytes(blob[offs[i]:offs[i + 1]]).decode()
    raise AssertionError("unreachable")


def _progress(n_records: int) -> None:
    # builders.py:257-258: every 500 000 records yielded
    for k in range(1, n_records // 500_000 + 1):
        print(f"\r[{k * 500_000:,} lines]", end="", file=sys.stderr)


def finalize(raw: RawResult, *, dtype: np.dtype, return_node_list: bool, raw_bytes_id: bool,
             verbose: bool, build_matrix: bool = True, path: Any = None):
    """Turn one native result into the reference's return value / warning / exception."""
    if raw.status in (nat.E_IO, nat.E_ARG, nat.E_DEVICE, nat.E_NOMEM, nat.E_UNSUPPORTED):
        raise_for_status(raw, dtype, path)
    if raw.status == nat.E_GZIP:  # the lines gzip returned before failing were parsed first
        if raw.has_warning:
            warnings.warn(f"Skipping unsupported record: {chr(raw.warn_byte)}", RuntimeWarning, stacklevel=3)
        if verbose:
            _progress(raw.n_records)
        raise_for_status(raw, dtype, path)
    if raw.has_warning:  # parser.py:124-130
        warnings.warn(f"Skipping unsupported record: {chr(raw.warn_byte)}", RuntimeWarning, stacklevel=3)
    parse_failed = nat.OK < raw.status < nat.E_CAST_OVERFLOW
    if verbose:
        _progress(raw.n_records_before_error if parse_failed else raw.n_records)
    if parse_failed:
        raise_for_status(raw, dtype, path)
    if verbose:
        print("\r[parse_gfa] done")
    if not build_matrix:
        return None
    raise_for_status(raw, dtype, path)  # dtype cast errors (after the parse loop)
    for _ in range(int(raw.n_cast_overflow)):  # numpy's per-element float32 cast warning
        warnings.warn("overflow encountered in cast", RuntimeWarning, stacklevel=3)
    n = int(raw.n_nodes)
    if raw.format == "coo":
        A = sp.coo_matrix((raw.data, (raw.rows, raw.cols)), shape=(n, n), dtype=dtype)
    else:
        A = sp.csr_matrix((raw.data, raw.indices, raw.indptr), shape=(n, n), dtype=dtype)
        if raw.indptr.dtype == np.int64 and A.indptr.dtype != np.int64:
            # scipy's own result keeps int64 here (coo.tocsr of more than 2^31 - 1 triplets sizes its
            # arrays by the triplets; the constructor's content check would narrow them)
            A.indices, A.indptr = raw.indices, raw.indptr
    if return_node_list:
        return A, _node_list(raw, raw_bytes_id)
    return A


def _dtype_of(dtype) -> np.dtype:
    dt = np.dtype(dtype)
    if dt.name not in nat.DTYPE_CODES:
        raise NotImplementedError(
            f"dtype {dt} is not supported by the GPU path (supported: {', '.join(nat.DTYPE_CODES)})")
    return dt


def _unit_dtype(dtype) -> np.dtype | None:
    """A dtype outside the five the kernels compute in, for a build whose every value is dtype(1.0) (no
    weight tag: builders.py:224-228 appends 1.0): the build then runs in int32 and its values — copy counts
    k of each entry (the SUM CSR's k, MAX-SYM's max(k_A, k_AT): builders.py:282-283) — become the sum of
    k ones in that dtype (_unit_values).  None for the five native dtypes."""
    dt = np.dtype(dtype)
    return None if dt.name in nat.DTYPE_CODES else dt


def _unit_values(counts: np.ndarray, dt: np.dtype) -> np.ndarray:
    """The sum of k ones in dtype dt for each copy count k (scipy sums duplicates in the matrix dtype):
    k itself while it is exact; an integer dtype whose sums would wrap raises NotImplementedError (a
    documented limit); scipy.sparse's own dtype check raises first for what it does not support."""
    sp.coo_matrix((np.zeros(0, dtype=dt), (np.zeros(0, np.int32), np.zeros(0, np.int32))), shape=(1, 1))
    k = np.asarray(counts)
    if k.size and dt.kind in "iu" and int(k.max()) > np.iinfo(dt).max:
        raise NotImplementedError(f"copy counts up to {int(k.max())} wrap in {dt}: not supported by the GPU path")
    return k.astype(dt)


def _with_unit_dtype(out, dt: np.dtype, return_node_list: bool):
    """An int32 unit-valued build's result in dtype dt (values: _unit_values of its copy counts)."""
    A = out[0] if return_node_list else out
    if A.format == "coo":  # every value is dtype(1.0)
        A = sp.coo_matrix((_unit_values(np.ones(A.nnz, dtype=np.int32), dt), (A.row, A.col)), shape=A.shape)
    else:
        B = sp.csr_matrix((_unit_values(A.data, dt), A.indices, A.indptr), shape=A.shape)
        if A.indptr.dtype == np.int64 and B.indptr.dtype != np.int64:  # (finalize's index-dtype rule)
            B.indices, B.indptr = A.indices, A.indptr
        A = B
    return (A, out[1]) if return_node_list else A


def parse_gfa(
    path,
    *,
    build_graph: bool,
    build_matrix: bool,
    directed: bool = True,
    weight_tag: str | None = None,
    store_seq: bool = False,
    store_tags: bool = False,
    strip_orientation: bool = False,
    verbose: bool = False,
    bidirected: bool = False,
    keep_directed_bidir: bool = False,
    backend: str = "networkx",
    dtype: str | object = "float64",
    asymmetric: bool = False,
    raw_bytes_id: bool = False,
    return_node_list: bool = False,
    max_tag_mb: float = 100.0,
    split_on_alignment: bool = False,
    device: int = 0,
    shard: str = "never",
    chunk_bytes: int | None = None,
):
    """GPU ``parse_gfa`` (gfa2network/builders.py:30-299), matrix outputs only.

    Returns ``A`` or ``(A, node_list)`` exactly as the reference does for
    ``build_graph=False, build_matrix=True``.

    ``shard`` (extension; the reference has no such argument) decides only whether the ranks of a
    torch.distributed group split the file: ``"never"`` (default) builds on this process's GPU;
    with more than one rank, ``"auto"`` splits the file over the ranks (``parse_gfa_sharded``) when
    its working set would not fit a GPU's free HBM on some rank, ``"always"`` splits it regardless;
    both are collectives — every rank must make the same call on the same file (checked: a different
    path raises ValueError).  On this process's GPU, an input whose working set would not fit its
    free HBM — a plain file, a ``.gz`` (inflated on the host), stdin or a file object — is built in
    line-aligned chunks on that one GPU (``shard.build_chunked``: errors, cast errors and the
    one-shot warning come out as one piece would raise / emit them; the whole-matrix CSR is
    assembled in row bands when it does not fit either).  ``chunk_bytes`` (extension) forces that
    chunked build with chunks of about that many bytes.
    """
    if backend == "igraph":
        raise NotImplementedError("backend='igraph' is outside the GPU GFA->CSR path")
    if split_on_alignment:  # builders.py:110-128 (before the return_node_list check)
        if build_graph:
            raise NotImplementedError("graph objects (build_graph=True) are outside the GPU GFA->CSR path")
        return _parse_gfa_split(path, build_matrix=build_matrix, directed=directed, weight_tag=weight_tag,
                                strip_orientation=strip_orientation, bidirected=bidirected,
                                keep_directed_bidir=keep_directed_bidir, dtype=dtype, asymmetric=asymmetric,
                                raw_bytes_id=raw_bytes_id, return_node_list=return_node_list, device=device)
    if return_node_list and not build_matrix:  # builders.py:129-130
        raise ValueError("return_node_list requires build_matrix=True")
    if build_graph:
        raise NotImplementedError("graph objects (build_graph=True) are outside the GPU GFA->CSR path")
    ext = _unit_dtype(dtype) if build_matrix else None
    if ext is not None:  # another numpy dtype: unit values only, built in int32
        if weight_tag:
            raise NotImplementedError(f"dtype {ext} with a weight tag is not supported by the GPU path "
                                      f"(supported: {', '.join(nat.DTYPE_CODES)})")
        out = parse_gfa(path, build_graph=False, build_matrix=True, directed=directed, weight_tag=None,
                        strip_orientation=strip_orientation, verbose=verbose, bidirected=bidirected,
                        keep_directed_bidir=keep_directed_bidir, dtype="int32", asymmetric=asymmetric,
                        raw_bytes_id=raw_bytes_id, return_node_list=return_node_list, device=device, shard=shard,
                        chunk_bytes=chunk_bytes)
        return _with_unit_dtype(out, ext, return_node_list)
    dt = _dtype_of(dtype) if build_matrix else np.dtype("float64")
    if shard not in ("auto", "always", "never"):
        raise ValueError("shard must be 'auto', 'always' or 'never'")
    if build_matrix and _want_shard(path, shard, device):
        return parse_gfa_sharded(path, directed=directed, weight_tag=weight_tag, strip_orientation=strip_orientation,
                                 verbose=verbose, bidirected=bidirected, keep_directed_bidir=keep_directed_bidir,
                                 dtype=dt.name, asymmetric=asymmetric, raw_bytes_id=raw_bytes_id,
                                 return_node_list=return_node_list, device=device)
    src = path
    if build_matrix:  # one GPU, an input past its working set: chunks of it (any input kind)
        done, src = _one_gpu_chunked(path, chunk_bytes, device, directed=directed, weight_tag=weight_tag,
                                     verbose=verbose, bidirected=bidirected, keep_directed_bidir=keep_directed_bidir,
                                     strip_orientation=strip_orientation, dt=dt, asymmetric=asymmetric,
                                     raw_bytes_id=raw_bytes_id, return_node_list=return_node_list)
        if done is not None:
            return done
    opts = nat.make_options(
        directed=directed, bidirected=bidirected, keep_directed_bidir=keep_directed_bidir,
        asymmetric=asymmetric, strip_orientation=strip_orientation, dtype=dt.name,
        weight_tag=weight_tag or None, output=nat.OUT_PARSE,
        want_node_names=bool(return_node_list), device=device)
    raw = _run(src, opts)
    return finalize(raw, dtype=dt, return_node_list=return_node_list, raw_bytes_id=raw_bytes_id,
                    verbose=verbose, build_matrix=build_matrix, path=path)


def _parse_gfa_split(path, *, build_matrix: bool, directed: bool, weight_tag, strip_orientation: bool,
                     bidirected: bool, keep_directed_bidir: bool, dtype, asymmetric: bool, raw_bytes_id: bool,
                     return_node_list: bool, device: int, build=None):
    """``parse_gfa(..., split_on_alignment=True)`` matrix outputs (builders.py:302-568).

    1. The input is parsed on the GPU as the plain path parses it: every parser error, the
       one-shot unsupported-record warning and gzip failures are the reference's (its split
       path runs the same GFAParser loop over the whole input first, builders.py:330-346).
    2. ``g2n_split_render`` (csrc/g2n_split.cpp) cuts the segments at the E/C coordinates,
       re-targets the records (builders.py:348-430) and renders that record stream as GFA text;
       the ">10x" and "skipping ..." warnings are emitted here in the reference's order.
    3. The GPU builds the rendered stream with the caller's options (builders.py:460-557: the
       same matrix loop, COO, ``A.maximum(A.T)`` and node list).  Bidirected: the interval
       segments mint their plain keys first (builders.py:474-476), ahead of the GPU's nodes.
    verbose prints nothing on this path for matrix outputs (builders.py:536-537 is graph-only).
    ``build(src, mode, want_names) -> RawResult`` runs one build (default: the GPU through the
    C-ABI; src is a path or bytes) — the CPU tests pass the oracle as the checker.
    """
    dt = _dtype_of(dtype) if build_matrix else np.dtype("float64")
    if build is None:
        def build(src, mode: dict, want_names: bool):
            o = nat.make_options(output=nat.OUT_PARSE, want_node_names=want_names, device=device,
                                 **{k: v for k, v in mode.items() if k != "dtype"}, dtype=mode.get("dtype", "float64"))
            return nat.build_from_path(src, o) if isinstance(src, str) else nat.build_from_buffer(src, o)
    data = None
    if hasattr(path, "read"):
        data = path.read()
    elif str(path) == "-":
        data = sys.stdin.buffer.read()
    else:
        p = str(path)
        try:
            with open(p, "rb") as fh:
                blob = fh.read()
        except OSError:
            blob = None  # the build raises the reference's OSError
        if blob is not None and p.endswith(".gz"):
            try:
                data, _ = nat.gunzip(blob)
            except nat.GzipFailure:
                data = None  # corrupt gzip: the plain path's prefix semantics decide
        else:
            data = blob
    raw0 = build(str(path) if data is None else data, {"asymmetric": True}, False)
    finalize(raw0, dtype=np.dtype("float64"), return_node_list=False, raw_bytes_id=raw_bytes_id, verbose=False,
             build_matrix=False, path=path)
    if raw0.status != nat.OK:
        raise_for_status(raw0, np.dtype("float64"), path)
    del raw0
    text, blob, offs, warns, many, per_seg = nat.split_render(data, bidirected)
    if many:
        warnings.warn("split-on-alignment created >10x more nodes", RuntimeWarning, stacklevel=3)
    for kind, seg in warns:
        if kind == 0:
            warnings.warn(f"skipping edge with undefined coordinates on segment {seg.decode()}", RuntimeWarning,
                          stacklevel=3)
        else:
            warnings.warn(f"skipping link with undefined segment {seg.decode()}", RuntimeWarning, stacklevel=3)
    if not build_matrix:
        return None
    raw = build(text, dict(directed=directed, bidirected=bidirected, keep_directed_bidir=keep_directed_bidir,
                           asymmetric=asymmetric, strip_orientation=strip_orientation, dtype=dt.name,
                           weight_tag=weight_tag or None), bool(return_node_list))
    m = len(offs) - 1
    if bidirected and raw.status == nat.OK and m:
        # builders.py:348-377 + 460-476: segment s's records are its k intervals (plain keys), then
        # its k - 1 chain links, which mint its 2k oriented keys (k with keep_directed_bidir) in
        # the GPU's order; the edges' keys follow.  So GPU node g of block s moves to
        # (nodes before s) + k + (g - its block start): a monotonic map.
        n_gpu = int(raw.n_nodes)
        k = per_seg.astype(np.int64)
        c = np.where(k >= 2, k if keep_directed_bidir else 2 * k, 0)
        if m + n_gpu >= 2 ** 31:
            raise NotImplementedError("more than 2**31-1 nodes")
        gmap = np.arange(n_gpu, dtype=np.int64) + m
        blk_start = np.concatenate([[0], np.cumsum(c)])[:-1]
        before = np.concatenate([[0], np.cumsum(k + c)])[:-1]
        n_blk = int(c.sum())
        seg_of_g = np.repeat(np.arange(len(k)), c)
        gmap[:n_blk] = before[seg_of_g] + k[seg_of_g] + (np.arange(n_blk) - blk_start[seg_of_g])
        gmap = gmap.astype(np.int32)
        n_fin = m + n_gpu
        if raw.format == "coo":
            raw.rows = gmap[raw.rows]
            raw.cols = gmap[raw.cols]
        else:
            cnt = np.zeros(n_fin, dtype=np.int64)
            cnt[gmap] = np.diff(raw.indptr.astype(np.int64))
            raw.indptr = np.concatenate([[0], np.cumsum(cnt)]).astype(raw.indptr.dtype)
            raw.indices = gmap[raw.indices]
        if return_node_list:
            gb = raw.names_blob if raw.names_blob is not None else np.zeros(0, dtype=np.uint8)
            go = raw.names_offsets if raw.names_offsets is not None else np.zeros(1, dtype=np.int64)
            # final node p: the next interval segment name (host blob, in order) where no GPU node
            # lands, else GPU node g with gmap[g] = p — one gather over the two blobs (no per-name
            # Python objects)
            is_gpu = np.zeros(n_fin, dtype=bool)
            is_gpu[gmap] = True
            order = np.empty(n_fin, dtype=np.int64)
            order[~is_gpu] = np.arange(m, dtype=np.int64)
            order[gmap] = m + np.arange(n_gpu, dtype=np.int64)
            hb = np.asarray(blob, dtype=np.uint8)[:int(offs[m])] if m else np.zeros(0, dtype=np.uint8)
            src = np.concatenate([hb, np.asarray(gb, dtype=np.uint8)])
            src_offs = np.concatenate([np.asarray(offs[:m + 1], dtype=np.int64),
                                       np.asarray(go[1:], dtype=np.int64) + int(offs[m])])
            raw.names_blob, raw.names_offsets = nat.gather_names(src, src_offs, order)
        raw.n_nodes = n_fin
    elif not bidirected and return_node_list and raw.status == nat.OK and raw.names_offsets is None:
        raw.names_blob, raw.names_offsets = np.zeros(0, dtype=np.uint8), np.zeros(1, dtype=np.int64)
    return finalize(raw, dtype=dt, return_node_list=return_node_list, raw_bytes_id=raw_bytes_id, verbose=False,
                    path=path)


def _dist_world() -> int:
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover - torch is in the image
        return 1
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def _gz_inflated_estimate(p: str, size: int) -> int:
    """Bytes a .gz inflates to, for the shard decision: the last member's ISIZE (RFC 1952: the
    length mod 2^32) or 4x the compressed size (GFA text compresses 3-4x), whichever is larger."""
    try:
        with open(p, "rb") as fh:
            fh.seek(max(size - 4, 0))
            isize = int.from_bytes(fh.read(4), "little")
    except OSError:
        isize = 0
    return max(isize, 4 * size)


def _free_hbm(device: int, need: int = 0) -> int | None:
    """Free HBM of `device` (hipMemGetInfo through the C-ABI: no torch on the one-GPU path); None
    without such a device (the build itself then raises G2N_E_DEVICE).  When that is less than `need`,
    the host entry points' cached buffers (an earlier build's arena, g2n_release_shared) are released
    first and the free HBM read again: a cache must not send a build that fits to the chunked route."""
    try:
        free = nat.device_memory(device)[0]
        if free < need and nat.release_shared(device):
            free = nat.device_memory(device)[0]
        return free
    except RuntimeError:
        return None


def _chunk_plan(size: int, device: int) -> int:
    """The chunk size that lets an input of `size` bytes whose working set (WORKING_SET_PER_INPUT_BYTE
    x its size) exceeds the GPU's free HBM be built on this GPU alone (shard.build_chunked), or 0 (the
    one-piece build): each chunk's working set is then about half the free HBM."""
    free = _free_hbm(device, need=size * WORKING_SET_PER_INPUT_BYTE)
    if free is None or size * WORKING_SET_PER_INPUT_BYTE <= free:
        return 0
    return max(1 << 26, int(free // (2 * WORKING_SET_PER_INPUT_BYTE)))


class _Bytes:
    """Input already read into host memory, handed to the one-piece build as a file object."""

    def __init__(self, arr):
        self.arr = arr

    def read(self):
        return self.arr


def _one_gpu_chunked(path, chunk_bytes, device: int, **kw):
    """parse_gfa's one-GPU route for an input past the GPU's working set (any input kind the
    reference reads, parser.py:95-112): (the result, None) when it was built in chunks, else (None,
    the input for the one-piece build).  A plain file is measured on disk and its chunks pread;
    stdin and file objects are read into host memory first (the one-piece build would read them
    whole too); a ``.gz`` whose inflated size (last ISIZE, or 4x the compressed bytes) may not fit is
    inflated on the host (member-parallel / chunk-parallel, g2n_gunzip) and chunked from there — one
    that does not inflate cleanly goes to the one-piece build, whose exact reader raises gzip.py's
    error after the lines before it.  `chunk_bytes` (extension) forces chunks of about that size."""
    from .shard import FileSource, HostSource

    if hasattr(path, "read") or str(path) == "-":
        data = path.read() if hasattr(path, "read") else sys.stdin.buffer.read()
        arr = data if isinstance(data, np.ndarray) else np.frombuffer(data, dtype=np.uint8)
        cb = chunk_bytes or _chunk_plan(len(arr), device)
        if cb:
            return _parse_gfa_chunked(HostSource(arr), cb, device=device, path=path, **kw), None
        return None, _Bytes(arr)
    p = str(path)
    if not os.path.isfile(p):
        return None, path  # the one-piece build raises the reference's OSError
    size = os.path.getsize(p)
    if p.endswith(".gz"):
        free = None if chunk_bytes else _free_hbm(device, need=_gz_inflated_estimate(p, size) * WORKING_SET_PER_INPUT_BYTE)
        if not chunk_bytes and (free is None or _gz_inflated_estimate(p, size) * WORKING_SET_PER_INPUT_BYTE <= free):
            return None, path
        with open(p, "rb") as fh:
            blob = fh.read()
        try:
            data, _ = nat.gunzip(blob)
        except nat.GzipFailure:
            return None, path
        del blob
        arr = np.frombuffer(data, dtype=np.uint8)
        cb = chunk_bytes or _chunk_plan(len(arr), device)
        if cb:
            return _parse_gfa_chunked(HostSource(arr), cb, device=device, path=path, **kw), None
        return None, _Bytes(arr)
    cb = chunk_bytes or _chunk_plan(size, device)
    if cb:
        return _parse_gfa_chunked(FileSource(p), cb, device=device, path=path, **kw), None
    return None, path


def _parse_gfa_chunked(source, chunk_bytes: int, *, directed: bool, weight_tag, verbose: bool, bidirected: bool,
                       keep_directed_bidir: bool, strip_orientation: bool, dt, asymmetric: bool, raw_bytes_id: bool,
                       return_node_list: bool, device: int, engine=None, path=None, free_hbm=None, bands=None):
    """parse_gfa on one GPU in chunks of the input (shard.build_chunked; source: a path, FileSource or
    HostSource), or None past 2^31 - 1 nodes (the one-piece build reports that limit).  Errors and the
    warning come out as the one-piece build's (finalize).  The engine — two build contexts and their
    grow-only arenas — lives for this call only unless the caller passes one."""
    from .shard import HipEngine, _np, build_chunked, scipy_index_dtype

    gd = keep_directed_bidir or (not bidirected and directed)  # builders.py:143
    maxsym = gd and not asymmetric                               # builders.py:282
    eng = engine or HipEngine(device, torch_buffers=False)  # one GPU, no collective: no torch on this path
    try:
        res = build_chunked(source, engine=eng, chunk_bytes=chunk_bytes, directed=directed, bidirected=bidirected,
                            keep_directed_bidir=keep_directed_bidir, asymmetric=asymmetric,
                            strip_orientation=strip_orientation, dtype=dt.name, weight_tag=weight_tag or None,
                            gather_names=return_node_list, keep_coo=not maxsym, free_hbm=free_hbm, bands=bands)
        if res is None:
            return None
        raw = RawResult(status=res.status, err_line=res.err_line, err_index=res.err_index, err_value=res.err_value,
                        err_detail=res.err_detail, has_warning=res.has_warning, warn_byte=res.warn_byte,
                        warn_line=res.warn_line, n_lines=res.n_lines, n_records=res.n_records,
                        n_records_before_error=res.n_records_before_error, n_nodes=res.n_nodes, dtype=dt,
                        n_cast_overflow=res.n_cast_overflow)
        if res.status == 0:
            if not maxsym:  # parse_gfa's stream-order COO (builders.py:281)
                raw.format = "coo"
                idt = scipy_index_dtype(0, res.n_nodes)
                raw.rows = _np(res.coo[0]).astype(idt, copy=False)
                raw.cols = _np(res.coo[1]).astype(idt, copy=False)
                raw.data = _np(res.coo[2])
            else:
                raw.format = "csr"
                idt = scipy_index_dtype(res.index_maxval, res.n_nodes)
                raw.indptr = _np(res.indptr).astype(idt, copy=False)
                raw.indices = _np(res.indices).astype(idt, copy=False)
                raw.data = _np(res.data)
            if return_node_list:
                raw.names_blob, raw.names_offsets = res.names_blob, res.names_offsets
    finally:
        if engine is None:
            eng.close()
    return finalize(raw, dtype=dt, return_node_list=return_node_list, raw_bytes_id=raw_bytes_id, verbose=verbose,
                    path=path if path is not None else getattr(source, "path", None))


def _want_shard(path, shard: str, device: int) -> bool:
    """Split the file over the process group?  Only for a file on disk, more than one rank, and
    ("auto") a working set beyond a GPU's free HBM.  "auto" and "always" are collectives: the
    ranks agree on the path (every rank must pass the same file) and, for "auto", on the verdict
    (all-reduce MAX of the per-rank "does not fit" flags), so no rank enters the sharded build
    alone."""
    if shard == "never" or _dist_world() < 2:
        return False
    import torch
    import torch.distributed as dist

    here = not hasattr(path, "read") and str(path) != "-" and os.path.isfile(str(path))
    need = 0
    if here and shard == "always":
        need = 1
    elif here:
        p = str(path)
        size = os.path.getsize(p)
        work = (_gz_inflated_estimate(p, size) if p.endswith(".gz") else size) * WORKING_SET_PER_INPUT_BYTE
        free = _free_hbm(device, need=work)
        need = int(free is not None and work > free)
    ident = zlib.crc32(os.fsencode(os.path.abspath(str(path)))) if here else 0
    size = os.path.getsize(str(path)) if here else -1
    nccl = dist.get_backend() == "nccl"
    t = torch.tensor([need, ident, size, -ident, -size, int(here), -int(here)], dtype=torch.int64,
                     device=torch.device("cuda", torch.cuda.current_device()) if nccl else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    v = t.tolist()
    same = v[1] == -v[3] and v[2] == -v[4] and v[5] == -v[6]
    if v[5] and not same:
        raise ValueError(f"parse_gfa(shard={shard!r}) is a collective: every rank must pass the same file")
    return bool(v[5]) and bool(v[0])


def parse_gfa_sharded(path, *, directed: bool = True, weight_tag: str | None = None,
                      strip_orientation: bool = False, verbose: bool = False, bidirected: bool = False,
                      keep_directed_bidir: bool = False, dtype="float64", asymmetric: bool = False,
                      raw_bytes_id: bool = False, return_node_list: bool = False, output: str = "parse",
                      group=None, engine=None, root=None, device=None):
    """``parse_gfa(path, build_graph=False, build_matrix=True, ...)`` with the file split over the
    ranks of a torch.distributed group — a collective: every rank calls it with
    the same path.  Each rank preads only its line-aligned byte range (``file_line_ranges``) into
    its GPU's HBM, the ranks reconcile node ids (the decimal-id fast path or the general owner
    protocol, gfa2network_amd/shard.py) and route triplets to row owners.  The result — what
    parse_gfa returns (the MAX-SYM CSR, or the stream-order COO), or with ``output="csr"`` what
    ``convert_format(parse_gfa(...), "csr")`` returns — is assembled on every rank (``root=None``)
    or on rank ``root`` only (the other ranks return None; a failed build raises on every rank).
    ``device``: this rank's GPU (default: torch's current device) — the one ``shard="auto"`` measured.  Index dtypes follow scipy (int64 once
    the entries pass 2^31 - 1).  Exceptions, the one-shot warning and the verbose strings are the
    reference's (builders.py:95-299).  A multi-member / BGZF ``.gz`` is inflated member-wise: each
    rank inflates the members that start in its share of the compressed bytes and one all-to-all
    moves the text to the line-aligned ranges (``shard.gz_rank_text``); a file that does not split
    into clean member chains (one member, damage) is inflated by every rank, and one that does not
    inflate cleanly is built by every rank on its own GPU through the single-GPU path, whose gzip
    errors and prefix semantics are the reference's."""
    import torch

    from .shard import HipEngine, build_sharded, file_line_ranges, gather_coo, gather_csr, scipy_index_dtype

    dt = _dtype_of(dtype)
    if output not in ("parse", "csr"):
        raise ValueError("output must be 'parse' or 'csr'")
    import torch.distributed as dist

    def dev() -> int:  # this rank's GPU, resolved only where a GPU is used (CPU engines have none)
        if device is not None:
            return device
        d = getattr(engine, "device_index", None)
        return torch.cuda.current_device() if d is None else d

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    p = str(path)
    gd = keep_directed_bidir or (not bidirected and directed)  # builders.py:143
    maxsym = gd and not asymmetric                               # builders.py:282
    if p.endswith(".gz"):
        from .shard import gz_rank_text, line_ranges

        eng = engine or HipEngine(dev())
        got = gz_rank_text(p, eng, group)  # each rank inflates the members in its share of the bytes
        if got is not None:
            buf = got[0]
        else:  # not a clean member chain in slices (one member, damage): the whole file on every rank
            with open(p, "rb") as fh:
                blob = fh.read()
            try:
                data, _ = nat.gunzip(blob)
            except nat.GzipFailure:
                del blob
                opts = nat.make_options(directed=directed, bidirected=bidirected,
                                        keep_directed_bidir=keep_directed_bidir, asymmetric=asymmetric,
                                        strip_orientation=strip_orientation, dtype=dt.name,
                                        weight_tag=weight_tag or None,
                                        output=nat.OUT_CSR if output == "csr" else nat.OUT_PARSE,
                                        want_node_names=bool(return_node_list), device=dev())
                raw = _run(p, opts)  # the exact reader raises gzip.py's error after the prefix's lines
                out = finalize(raw, dtype=dt, return_node_list=return_node_list, raw_bytes_id=raw_bytes_id,
                               verbose=verbose, path=path)
                return out if root is None or rank == root else None
            del blob
            lo, hi = line_ranges(data, world)[rank]
            buf = torch.from_numpy(np.frombuffer(data, dtype=np.uint8)[lo:hi].copy()).to(eng.device)
            del data
    else:
        eng = engine or HipEngine(dev())
        lo, hi = file_line_ranges(p, world)[rank]
        buf = eng.read_range(p, lo, hi - lo)
    res = build_sharded(buf, engine=eng, group=group, directed=directed, bidirected=bidirected,
                        keep_directed_bidir=keep_directed_bidir, asymmetric=asymmetric,
                        strip_orientation=strip_orientation, dtype=dt.name, weight_tag=weight_tag or None,
                        gather_names=return_node_list, keep_coo=not maxsym and output == "parse", names_root=root,
                        trim=True)  # (a sharded file is one too large for a GPU: free each stage's dead buffers)
    del buf
    raw = RawResult(status=res.status, err_line=res.err_line, err_index=res.err_index, err_value=res.err_value,
                    err_detail=res.err_detail, has_warning=res.has_warning, warn_byte=res.warn_byte,
                    warn_line=res.warn_line, n_lines=res.n_lines, n_records=res.n_records,
                    n_records_before_error=res.n_records_before_error, n_nodes=res.n_nodes, dtype=dt,
                    n_cast_overflow=res.n_cast_overflow)
    if res.status == 0:
        if not maxsym and output == "parse":
            raw.format = "coo"
            got = gather_coo(res, group, root)
            if got is not None:
                raw.rows, raw.cols, raw.data = got
                idt = scipy_index_dtype(0, res.n_nodes)
                raw.rows, raw.cols = raw.rows.astype(idt, copy=False), raw.cols.astype(idt, copy=False)
        else:
            raw.format = "csr"
            got = gather_csr(res, group, root)
            if got is not None:
                raw.indptr, raw.indices, raw.data = got
        if root is not None and rank != root:
            return None
        if return_node_list:
            raw.names_blob, raw.names_offsets = res.names_blob, res.names_offsets
    elif root is not None and rank != root:
        # a failed build (every rank agrees on its status) raises on every rank, not only on the
        # root: None means success.  The warnings and verbose strings stay the root's.
        import warnings

        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            finalize(raw, dtype=dt, return_node_list=False, raw_bytes_id=raw_bytes_id, verbose=False, path=path)
        raise AssertionError(f"sharded build status {res.status} did not raise")  # finalize raises on any error
    return finalize(raw, dtype=dt, return_node_list=return_node_list, raw_bytes_id=raw_bytes_id, verbose=verbose,
                    path=path)


def parse_gfa_names(path, *, raw_bytes_id: bool = False, **kw):
    """``parse_gfa(path, build_graph=False, build_matrix=True, return_node_list=True, ...)`` for
    writers that never need the Python list (the convert CLI): returns ``(A, blob, offsets)``, the
    node names as the library's blob + offsets in id order.  A name that is not UTF-8 raises
    here unless raw_bytes_id, exactly where building the list would (builders.py:284-288)."""
    if kw.get("backend", "networkx") == "igraph":
        raise NotImplementedError("backend='igraph' is outside the GPU GFA->CSR path")
    if kw.pop("build_graph", False):
        raise NotImplementedError("graph objects (build_graph=True) are outside the GPU GFA->CSR path")
    if kw.pop("split_on_alignment", False):  # cli.py:111-115 --split-on-alignment: through the list
        A, nodes = parse_gfa(path, build_graph=False, build_matrix=True, return_node_list=True,
                             split_on_alignment=True, raw_bytes_id=raw_bytes_id, **kw)
        enc = [x if raw_bytes_id else x.encode() for x in nodes]
        offs = np.zeros(len(enc) + 1, dtype=np.int64)
        offs[1:] = np.cumsum([len(x) for x in enc], dtype=np.int64)
        return A, np.frombuffer(b"".join(enc), dtype=np.uint8), offs
    for k in ("store_seq", "store_tags", "max_tag_mb", "backend"):
        kw.pop(k, None)
    verbose = kw.pop("verbose", False)
    device = kw.pop("device", 0)
    dt = _dtype_of(kw.pop("dtype", "float64"))
    wt = kw.pop("weight_tag", None)
    opts = nat.make_options(dtype=dt.name, weight_tag=wt or None, output=nat.OUT_PARSE, want_node_names=True,
                            device=device, **kw)
    raw = _run(path, opts)
    A = finalize(raw, dtype=dt, return_node_list=False, raw_bytes_id=raw_bytes_id, verbose=verbose, path=path)
    blob, offs = raw.names_blob, raw.names_offsets
    if offs is None:
        offs = np.zeros(1, dtype=np.int64)
        blob = np.zeros(0, dtype=np.uint8)
    if not raw_bytes_id:
        bad = nat.first_bad_utf8(blob, offs)
        if bad >= 0:
            bytes(blob[offs[bad]:offs[bad + 1]]).decode()
            raise AssertionError("decode of the reported name unexpectedly succeeded")
    return A, blob, offs


def _run(path, opts) -> RawResult:
    """GFAParser's source rules (parser.py:95-112): file object, '-' = stdin, else a path."""
    if hasattr(path, "read"):
        return nat.build_from_buffer(path.read(), opts)
    p = str(path)
    if p == "-":
        return nat.build_from_buffer(sys.stdin.buffer.read(), opts)
    return nat.build_from_path(p, opts)


def export_edge_list(gfa, output="-", *, bidirected: bool = False, device: int = 0) -> None:
    """``gfa2network export GFA --format edge-list [--bidirected] --output PATH`` (cli.py:264-281).

    One ``u\tv`` line per L/E/C record in stream order (bidirected: ``u:ori\tv:ori``), the
    record keys the reference's parser yields (parser.py:206-341), rendered on the GPU from the
    same parse as the matrix path (``G2N_OUT_EDGE_LIST``).  Failure behaviour follows the
    reference's streaming loop: the output file is opened first, the lines of the records
    before a failing one are written, then the failure is raised (a malformed record, the
    ``u.decode()`` / ``v.decode()`` of a key that is not UTF-8, or a gzip error after the lines
    gzip returned); the unsupported-record warning is emitted as by ``GFAParser``.
    """
    opts = nat.make_options(bidirected=bidirected, output=nat.OUT_EDGE_LIST, device=device)
    fh = open(output, "wb") if output != "-" else None  # cli.py:266-267: opened before parsing
    try:
        src = gfa
        if not hasattr(gfa, "read") and str(gfa) == "-":
            src = io.BytesIO(sys.stdin.buffer.read())  # parser.py:104: sys.stdin.buffer, not gunzipped
        if hasattr(src, "read"):
            raw = nat.build_from_buffer(src.read(), opts)
        else:
            raw = nat.build_from_path(str(src), opts)
        if raw.has_warning:  # parser.py:124-130
            warnings.warn(f"Skipping unsupported record: {chr(raw.warn_byte)}", RuntimeWarning, stacklevel=2)
        # on a failure the text holds the lines the reference wrote before it: the records before
        # a malformed line, before an undecodable key, or before the gzip error (the lines gzip
        # returned) — rendered by the native build from the input it already holds
        text = raw.data if raw.format == "text" and raw.data is not None else np.zeros(0, np.uint8)
        if fh is not None:
            fh.write(memoryview(text))
        else:
            sys.stdout.flush()
            sys.stdout.buffer.write(memoryview(text))
            sys.stdout.buffer.flush()
        raise_for_status(raw, np.dtype("bool"), gfa)
    finally:
        if fh is not None:
            fh.close()


def _keep_index_dtype(M, raw):
    """scipy's coo.tocsr() / tocsc() past 2^31 - 1 COO entries keeps int64 indptr / indices even when
    summing duplicates leaves fewer entries (_coo_to_compressed sizes by coo.nnz); the compressed
    constructor's content check alone would narrow them."""
    if raw.indptr.dtype == np.int64 and M.indptr.dtype != np.int64:
        M.indices, M.indptr = raw.indices, raw.indptr
    return M


def _coo_data(A):
    """The COO's values as the kernels take them: a dtype outside the native five only when every value
    is 1 (then int32 ones, the sums mapped back by _unit_values), else NotImplementedError."""
    ext = _unit_dtype(A.dtype)
    if ext is None:
        return A.data, None
    if not bool(np.all(A.data == 1)):
        raise NotImplementedError(f"GPU COO->CSR of dtype {ext} takes unit values only "
                                  f"(any values: {', '.join(nat.DTYPE_CODES)})")
    return np.ones(len(A.data), dtype=np.int32), ext


def _native_tocsr(A, device: int = 0):
    """scipy coo.tocsr() on the GPU: duplicates summed in dtype in scipy's order."""
    n_rows, n_cols = A.shape
    data, ext = _coo_data(A)
    raw = nat.coo_to_csr(A.row, A.col, data, n_rows, n_cols, device)
    vals = raw.data if ext is None else _unit_values(raw.data, ext)
    return _keep_index_dtype(sp.csr_matrix((vals, raw.indices, raw.indptr), shape=A.shape, dtype=A.dtype), raw)


def _native_tocsc(A, device: int = 0):
    """scipy coo.tocsc(): the CSR of the transposed coordinates, read as CSC."""
    n_rows, n_cols = A.shape
    data, ext = _coo_data(A)
    raw = nat.coo_to_csr(A.col, A.row, data, n_cols, n_rows, device)
    vals = raw.data if ext is None else _unit_values(raw.data, ext)
    return _keep_index_dtype(sp.csc_matrix((vals, raw.indices, raw.indptr), shape=A.shape, dtype=A.dtype), raw)


def convert_format(A, fmt: str, *, verbose: bool = False):
    """GPU ``convert_format`` (gfa2network/utils.py:40-63)."""
    fmt = fmt.lower()
    if fmt not in {"csr", "csc", "coo", "dok"}:
        raise ValueError("matrix-format must be csr|csc|coo|dok")
    if fmt == "coo":
        return A
    if verbose:  # utils.py:49-53
        if _HAS_TQDM:
            bar = tqdm(total=1, bar_format="{desc} …{elapsed}", desc=f"[convert→{fmt}")
        else:
            start = time.perf_counter()
            print(f"[convert] -> {fmt} …", end="", file=sys.stderr, flush=True)
    if fmt == A.format:
        out = A
    elif fmt == "dok":
        # a Python dict of (row, col) -> value: scipy's own asformat("dok") on the GPU-built
        # matrix (for a COO it sums duplicates in place, in stream order, as the reference's
        # A.asformat(fmt) does, utils.py:55)
        out = A.asformat("dok")
    else:
        coo = A if A.format == "coo" else A.tocoo()
        out = _native_tocsr(coo) if fmt == "csr" else _native_tocsc(coo)
    if verbose:  # utils.py:56-62
        if _HAS_TQDM:
            bar.update(1)
            bar.close()
        else:
            print(f" done in {time.perf_counter() - start:,.1f}s", file=sys.stderr)
    return out


def save_matrix(A, dest: Path, *, verbose: bool = False, max_dense_gb: float = 5.0):
    """Writer of ``convert --matrix`` (gfa2network/utils.py:66-105): same guard and formats."""
    MAX_DENSE_BYTES = max_dense_gb * 1_000_000_000
    dest = Path(dest)
    if dest.suffix in {".csv", ".npy"}:
        nnz = A.nnz if sp.issparse(A) else A.size
        itemsize = A.dtype.itemsize if hasattr(A, "dtype") else 8
        if nnz * itemsize > MAX_DENSE_BYTES:
            raise MemoryError(
                f"dense export would allocate {nnz*itemsize/1e9:.1f} GB; choose a sparse .npz or write an edge list instead"
            )
    if verbose:  # utils.py:77-83
        msg = f"[save] {dest.suffix[1:]} → {dest}"
        if _HAS_TQDM:
            bar = tqdm(total=1, bar_format="{desc} …{elapsed}", desc=msg)
        else:
            start = time.perf_counter()
            print(msg, "...", end="", file=sys.stderr, flush=True)
    if dest.suffix == ".npz":
        save_npz(dest, A)
    elif dest.suffix == ".npy":
        np.save(dest, A.toarray() if sp.issparse(A) else A)
    elif dest.suffix == ".csv":
        np.savetxt(dest, A.toarray() if sp.issparse(A) else A, delimiter=",", fmt="%.6g")
    else:
        raise ValueError("matrix path must end with .npz, .npy, or .csv")
    if verbose:  # utils.py:99-105
        if _HAS_TQDM:
            bar.update(1)
            bar.close()
        else:
            print(f" done in {time.perf_counter() - start:,.1f}s", file=sys.stderr)


def _npy_header(val: np.ndarray) -> bytes:
    """The .npy header numpy.lib.format.write_array puts before val's bytes."""
    import io

    from numpy.lib import format as npf

    bio = io.BytesIO()
    npf._write_array_header(bio, npf.header_data_from_array_1_0(val), None)
    return bio.getvalue()


def save_npz(file, matrix, compressed: bool = True) -> None:
    """scipy.sparse.save_npz (scipy 1.15 _matrix_io.py, members in its order) with the zip written
    natively: members deflated on host threads (g2n_write_npz), numpy's zip64 layout; loads with
    scipy.sparse.load_npz / numpy.load.  Uncompressed or unsupported formats fall back to scipy."""
    fmt = matrix.format
    if not compressed or fmt not in ("csr", "csc", "bsr", "coo") or fmt == "bsr":
        sp.save_npz(file, matrix, compressed=compressed)
        return
    path = os.fspath(file)
    if not path.endswith(".npz"):  # numpy _savez
        path = path + ".npz"
    members = {}
    if fmt in ("csr", "csc"):
        members.update(indices=matrix.indices, indptr=matrix.indptr)
    else:
        members.update(row=matrix.row, col=matrix.col)
    members.update(format=fmt.encode("ascii"), shape=matrix.shape, data=matrix.data)
    if isinstance(matrix, sp.sparray):
        members.update(_is_array=True)
    out = []
    for key, val in members.items():
        val = np.asanyarray(val)
        if val.dtype.hasobject:
            sp.save_npz(file, matrix, compressed=compressed)
            return
        arr = val if val.flags.c_contiguous else np.ascontiguousarray(val)
        out.append((key + ".npy", _npy_header(val), arr.reshape(-1).view(np.uint8) if arr.size else arr))
    with open(path, "wb"):  # the reference's zipfile.ZipFile(path, "w") open: same OSError cases
        pass
    nat.write_npz(path, out, int(os.environ.get("G2N_NPZ_LEVEL", "-1")))


def save_node_map_native(blob: np.ndarray, offsets: np.ndarray, dest: Path, raw_bytes_id: bool) -> None:
    """save_node_map (utils.py:108-114) from the names blob, written on host threads.  raw_bytes_id:
    names are decoded while writing, so the first non-UTF-8 name raises after the lines before it
    were written, as in the reference."""
    with open(dest, "w"):  # the reference's open(dest, "w"): same OSError cases
        pass
    bad = nat.write_node_map(str(dest), blob, offsets, check_utf8=raw_bytes_id)
    if bad >= 0:
        bytes(blob[offsets[bad]:offsets[bad + 1]]).decode()
        raise AssertionError("decode of the reported name unexpectedly succeeded")


def save_node_map(nodes, dest: Path) -> None:
    """``<matrix>.nodes.tsv`` sidecar (gfa2network/utils.py:108-114): ``i\\tname\\n``."""
    with open(dest, "w") as fh:
        for i, node in enumerate(nodes):
            if isinstance(node, (bytes, bytearray)):
                node = node.decode()
            fh.write(f"{i}\t{node}\n")
