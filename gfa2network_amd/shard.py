"""Sharded build of ONE GFA file over the ranks of a torch.distributed group.

The reference parses one file on one core (`parser.py:114` line loop, `builders.py:190-234`
dict minting and triplets); its node ids are the order of first touch over the whole file.
Here each rank takes a contiguous, line-aligned byte range and the ranks reconcile:

1. local build (HIP, `g2n_build_device`, output COO): the range as a file of its own — a
   stream-order COO over LOCAL ids (first touch inside the range) and the local names;
2. names to owners (`g2n_partition_keys`, hash of the bytes mod G; all-to-all-v): an owner
   receives each key from every rank that has it, concatenated in rank order, each rank's keys
   in local-id order — i.e. in GLOBAL first-touch order, because ranges are contiguous;
3. owner dedup (`g2n_dedup_keys`, exact bytes, the GPU dictionary): the first occurrence of
   a key carries its order key (source rank, local id);
4. global ids: the owners' distinct order keys are all-gathered; a key's id is the number of
   distinct keys, over all owners, with a smaller order key (the reference's dict insertion
   order); ids go back to the source ranks (all-to-all-v) → local → global id map;
5. triplets to row owners (`g2n_route_triplets`, all-to-all-v; rank k owns rows
   [ceil(k n / G), ceil((k+1) n / G))), plus the A.T stream for MAX-SYM; arrivals are in global
   stream order, so scipy's duplicate-summation order is kept;
6. the rank's CSR row slice (`g2n_csr_from_coo_pair`): coo.tocsr() or A.maximum(A.T).

Fast path (decimal ids, the layout of vg / odgi / PGGB graphs with compacted ids and of the
synthetic configs): when the file's S lines come first and name their segments "1".."N" in
order, a node's global id is arithmetic on its name, so steps 2-4 collapse to an all-gather of
the ranges' record counts (each rank learns how many S lines precede it and N) and one
all-reduce of the ranges' verdicts ("every range's ids are global decimals"): each rank parses
its range straight into global ids (`g2n_build_device` with options.range_flags = G2N_RANGE_DECIMAL), routes the
triplets with an identity map and builds its slice.  Any range that breaks the premise (or
holds an error / warning / slow weight) makes every rank take the general protocol above.

Errors and the one-shot unsupported-record warning are resolved across ranks in stream
order (the earliest parse error wins; cast errors only when no rank has a parse error).

The exchange runs on torch tensors: device tensors with the nccl (RCCL) backend, host tensors
with gloo.  The per-rank compute goes through an engine: `HipEngine` (the product: libg2n.so
on this rank's GPU); tests drive the same protocol with a CPU engine built on the oracle.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

from . import _native as nat

TORCH_DTYPES = {"bool": "uint8", "int8": "int8", "int32": "int32", "float32": "float32", "float64": "float64"}
CAST_ERRORS = (10, 11, 12)  # G2N_E_CAST_*: raised by np.array(data, dtype) after the whole parse


@dataclass
class LocalShard:
    """One rank's range built on its own (local ids)."""

    status: int
    err_line: int
    err_index: int
    err_value: float
    err_detail: bytes
    warn_line: int  # first unsupported-record line of the range, -1 if none
    has_warning: bool
    warn_byte: int
    n_lines: int
    n_records: int
    n_records_before_error: int
    n_edges: int
    n_local_nodes: int
    rows: object = None  # torch int32, stream order
    cols: object = None
    data: object = None  # torch dtype per TORCH_DTYPES
    names_blob: object = None  # torch uint8
    names_offsets: object = None  # torch int64, n_local_nodes + 1
    n_cast_overflow: int = 0
    parse_path: str = ""  # build_decimal: "tile_local" (the one-pass lean parse) or "k1" (tile counts first)
    phase_ms: dict = field(default_factory=dict)  # the local build's device phases (hipEvents; diagnostics)
    # G2N_RANGE_SLOTS: rows / cols are the parse's group slots (device pointer of the per-group counts,
    # groups, entries per group) holding n_trip entries in all; None: rows / cols in stream order
    slots: tuple | None = None
    n_trip: int = -1

    def triplets(self) -> int:
        """The entries the COO holds (rows.numel(), unless it is in group slots)."""
        return self.n_trip if self.slots is not None else int(self.rows.numel())


@dataclass
class ShardResult:
    """This rank's slice of the global result (rows [row_lo, row_hi) of an n_nodes^2 CSR)."""

    status: int
    err_line: int = -1
    err_index: int = -1
    err_value: float = 0.0
    err_detail: bytes = b""
    has_warning: bool = False
    warn_byte: int = 0
    warn_line: int = -1
    n_lines: int = 0
    n_records: int = 0
    n_records_before_error: int = 0
    n_edges: int = 0
    n_nodes: int = 0
    row_lo: int = 0
    row_hi: int = 0
    indptr: object = None
    indices: object = None
    data: object = None
    names_blob: object = None  # node keys in id order (numpy uint8 blob + int64 offsets), when gather_names
    names_offsets: object = None
    index_maxval: int = 0  # what scipy sizes the result's index dtype by (scipy_index_dtype)
    n_cast_overflow: int = 0
    timings_ms: dict = field(default_factory=dict)
    fast_path: bool = False  # the decimal-id fast path built it
    parse_path: str = ""  # fast path: how this rank's range was parsed ("tile_local" or "k1")
    coo: tuple | None = None  # keep_coo: this range's stream-order triplets over global ids
    a2a_bytes_sent: int = 0  # bytes this rank's all-to-all-v calls sent to other ranks (diagnostics)
    coo_layout: str = ""  # fast path: "group_slots" (routed / assembled from the parse's slots) or "stream"

    @property
    def names(self) -> list | None:
        """The node keys in id order as a list of bytes (None unless gather_names)."""
        if self.names_offsets is None:
            return None
        b, o = self.names_blob, self.names_offsets
        return [bytes(b[o[i]:o[i + 1]]) for i in range(len(o) - 1)]


INT32_MAX = 2**31 - 1


def scipy_index_dtype(maxval: int, n: int):
    """The index dtype scipy gives the result (scipy 1.15 ``get_index_dtype(..., maxval,
    check_contents=True)`` in the csr / coo constructors): int64 once a count or the shape passes
    int32, else int32.  maxval: the MAX-SYM CSR's nnz (``csr_binop_csr`` result, builders.py:283);
    for coo.tocsr() the triplet count with duplicates (``_coo_to_compressed`` sizes indptr by
    ``max(coo.nnz, N)`` before summing, utils.py:55); 0 for the COO (shape only)."""
    return np.int64 if max(int(maxval), int(n)) > INT32_MAX else np.int32


def concat_indptr(parts, dtype) -> np.ndarray:
    """The full indptr from the row slices' local indptrs (each starting at 0), in ``dtype``."""
    n = sum(max(len(p) - 1, 0) for p in parts)
    out = np.zeros(n + 1, dtype=dtype)
    base, r = 0, 0
    for p in parts:
        p = np.asarray(p)
        k = len(p) - 1
        if k <= 0:
            continue
        out[r + 1:r + k + 1] = p[1:].astype(np.int64) + base
        base += int(p[-1])
        r += k
    return out


def line_ranges(data: bytes | np.ndarray, n_ranks: int) -> list[tuple[int, int]]:
    """Contiguous line-aligned byte ranges: range r starts at the first line start at or after
    r * len / G (the line holding that offset belongs to the range holding its first byte)."""
    buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    n = len(buf)
    starts = [0]
    for r in range(1, n_ranks):
        nominal = r * n // n_ranks
        s = nominal
        if 0 < s < n and buf[s - 1] != 0x0A:
            pos, win = s, 1 << 16  # growing windows: no scan past the next newline
            s = n
            while pos < n:
                nl = np.flatnonzero(buf[pos:pos + win] == 0x0A)
                if len(nl):
                    s = pos + int(nl[0]) + 1
                    break
                pos += win
                win = min(win * 2, 1 << 26)
        starts.append(max(s, starts[-1]))
    return [(starts[r], starts[r + 1] if r + 1 < n_ranks else n) for r in range(n_ranks)]


def file_line_ranges(path: str, n_ranks: int, window: int = 1 << 16) -> list[tuple[int, int]]:
    """line_ranges() of a file on disk without reading it whole: each boundary is found with
    os.pread windows from its nominal offset r * size / G (parser.py:114 lines, `\n` only)."""
    import os

    size = os.path.getsize(path)
    starts = [0]
    with open(path, "rb") as fh:
        fd = fh.fileno()
        for r in range(1, n_ranks):
            nominal = r * size // n_ranks
            s = nominal
            if 0 < s < size and os.pread(fd, 1, s - 1) != b"\n":
                pos = s
                while True:
                    chunk = os.pread(fd, window, pos)
                    k = chunk.find(b"\n")
                    if k >= 0:
                        s = pos + k + 1
                        break
                    if len(chunk) < window:
                        s = size
                        break
                    pos += len(chunk)
            starts.append(max(s, starts[-1]))
    return [(starts[r], starts[r + 1] if r + 1 < n_ranks else size) for r in range(n_ranks)]


# ------------------------------------------------------------------------ engines --
class DevArray:
    """A view of `n` elements of a device array owned by an engine context (no copy): valid until
    the next build on that context.  Exposes what the engine calls read (data_ptr, numel, [a:b])."""

    def __init__(self, ptr: int, n: int, itemsize: int):
        self.ptr, self.n, self.itemsize = ptr, n, itemsize

    def data_ptr(self):
        return self.ptr

    def numel(self):
        return self.n

    def __getitem__(self, sl: slice):
        a, b, _ = sl.indices(self.n)
        return DevArray(self.ptr + a * self.itemsize, max(b - a, 0), self.itemsize)


class _HostView:
    """What DevBuf.cpu() returns: .numpy() of the host copy (the torch-tensor idiom the protocol uses)."""

    def __init__(self, arr):
        self.arr = arr

    def numpy(self):
        return self.arr


class _HipAlloc:
    """One hipMalloc'd block, freed with the last DevBuf viewing it."""

    def __init__(self, hip, device: int, nbytes: int):
        self.hip, self.ptr = hip, ctypes.c_void_p()
        if hip.hipSetDevice(device) != 0:
            raise MemoryError(f"hipSetDevice({device}) failed")
        if hip.hipMalloc(ctypes.byref(self.ptr), max(int(nbytes), 16)) != 0:
            hip.hipGetLastError()
            # once more without the host entry points' cached buffers (g2n_release_shared)
            if not nat.release_shared(device) or hip.hipMalloc(ctypes.byref(self.ptr), max(int(nbytes), 16)) != 0:
                hip.hipGetLastError()
                self.ptr = ctypes.c_void_p()
                raise MemoryError(f"hipMalloc of {nbytes} bytes failed on device {device}")

    def __del__(self):
        try:
            if self.ptr:
                self.hip.hipFree(self.ptr)
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


class DevBuf:
    """A 1-D device array owned through the HIP runtime (hipMalloc / hipFree over ctypes) — the
    one-GPU chunked build's buffers without torch.  Exposes what the engine and
    the chunked code read: numel, data_ptr, element_size, dtype, 1-D slices (views), contiguous / to
    (itself), cpu().numpy() / numpy() / tolist() (host copies)."""

    def __init__(self, n: int, dtype, device: int = 0, _alloc=None, _ptr=None):
        self.dtype, self.n, self.device = np.dtype(dtype), int(n), device
        self.hip = nat.hip_runtime()
        self._alloc = _alloc if _alloc is not None else _HipAlloc(self.hip, device, self.n * self.dtype.itemsize)
        self.ptr = _ptr if _ptr is not None else self._alloc.ptr.value

    def numel(self):
        return self.n

    def data_ptr(self):
        return self.ptr

    def element_size(self):
        return self.dtype.itemsize

    def __len__(self):
        return self.n

    def __getitem__(self, sl: slice):
        a, b, step = sl.indices(self.n)
        if step != 1:
            raise IndexError("DevBuf: unit-stride slices only")
        return DevBuf(max(b - a, 0), self.dtype, self.device, self._alloc, self.ptr + a * self.dtype.itemsize)

    def contiguous(self):
        return self

    def to(self, device):
        return self

    def numpy(self) -> np.ndarray:
        out = np.empty(self.n, dtype=self.dtype)
        if self.n and self.hip.hipMemcpy(out.ctypes.data, self.ptr, out.nbytes, 2) != 0:  # device to host
            raise RuntimeError("hipMemcpy failed")
        return out

    def cpu(self):
        return _HostView(self.numpy())

    def tolist(self):
        return self.numpy().tolist()


class _HipKeyset:
    """g2n_keyset on an engine's context: add(blob, offsets) -> (ids int32 of the keys, keys in the set);
    names() -> the set's keys in id order (copies); close()."""

    def __init__(self, eng):
        self.eng = eng
        self.h = ctypes.c_void_p()
        eng._check(eng.lib.g2n_keyset_create(eng.ctx, ctypes.byref(self.h)), "g2n_keyset_create")

    def add(self, blob, offsets):
        eng = self.eng
        n = offsets.numel() - 1
        ids = eng._empty(max(n, 1), "int32")
        tot = ctypes.c_uint64(0)
        eng._sync()
        eng._check(eng.lib.g2n_keyset_add(self.h, blob.data_ptr() if blob.numel() else None, blob.numel(),
                                          offsets.data_ptr(), n, ids.data_ptr(), ctypes.byref(tot)), "g2n_keyset_add")
        return ids[:n], int(tot.value)

    def names(self):
        eng = self.eng
        pb, po, n, nb = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64(0), ctypes.c_uint64(0)
        eng._check(eng.lib.g2n_keyset_view(self.h, ctypes.byref(pb), ctypes.byref(po), ctypes.byref(n),
                                           ctypes.byref(nb)), "g2n_keyset_view")
        return eng._copy_out(pb.value, int(nb.value), "uint8"), eng._copy_out(po.value, int(n.value) + 1, "int64")

    def close(self):
        if self.h:
            self.eng.lib.g2n_keyset_free(self.h)
            self.h = ctypes.c_void_p()


class HipEngine:
    """The product engine: libg2n.so on one GPU; buffers are torch device tensors (or DevArray
    views of a context's arena) — or, torch_buffers=False (the one-GPU chunked build: no collective,
    so no torch), DevBuf arrays allocated through the HIP runtime."""

    supports_views = True
    supports_slots = True  # build_decimal_range(slots=True) / route_slots / csr_slots (G2N_RANGE_SLOTS)

    def __init__(self, device: int = 0, torch_buffers: bool = True):
        if torch_buffers:
            import torch

            self.torch = torch
            self.device = torch.device("cuda", device)
        else:
            self.torch = None
            self.device = device
        self.lib = nat.load()
        self.device_index = device
        self.ctx = self.lib.g2n_context_create(device)
        if not self.ctx:
            raise nat.NativeUnavailable(nat.last_error())
        self._hip = nat.hip_runtime()
        self.ctx_b = None  # the fast path's build context: its COO is read in place by route / csr (on ctx)

    def close(self):
        for name in ("ctx", "ctx_b"):
            if getattr(self, name):
                self.lib.g2n_context_destroy(getattr(self, name))
                setattr(self, name, None)

    def _sync(self):
        # (DevBuf work is synchronous — hipMemcpy, and every g2n call returns after its stream drained)
        if self.torch is not None:
            self.torch.cuda.current_stream(self.device).synchronize()

    def _check(self, rc: int, what: str):
        if rc != 0:
            raise RuntimeError(f"{what}: {nat.status_name(rc)}: {nat.last_error()}")

    def _empty(self, n, dtype: str):
        """n elements of numpy dtype name `dtype` on this GPU: a torch tensor or a DevBuf."""
        if self.torch is None:
            return DevBuf(n, dtype, self.device_index)
        return self.torch.empty(n, dtype=getattr(self.torch, dtype), device=self.device)

    def _copy_out(self, ptr, n, dtype: str):
        t = self._empty(n, dtype)
        nbytes = n * t.element_size()
        if nbytes:
            if self._hip.hipMemcpy(t.data_ptr(), ptr, nbytes, 3) != 0:  # device to device
                raise RuntimeError("hipMemcpy failed")
        return t

    def cat(self, xs):
        """1-D device arrays of one dtype, concatenated (torch.cat, or D2D copies into one DevBuf)."""
        if len(xs) == 1:
            return xs[0]
        if self.torch is not None:
            return self.torch.cat(xs)
        out = DevBuf(sum(x.numel() for x in xs), xs[0].dtype, self.device_index)
        pos = 0
        for x in xs:
            nb = x.numel() * x.element_size()
            if nb and self._hip.hipMemcpy(out.ptr + pos, x.data_ptr(), nb, 3) != 0:
                raise RuntimeError("hipMemcpy failed")
            pos += nb
        return out

    def empty(self, n, dtype):
        if self.torch is None or isinstance(dtype, str):
            return self._empty(n, dtype if isinstance(dtype, str) else str(dtype).replace("torch.", ""))
        return self.torch.empty(n, dtype=dtype, device=self.device)

    def trim(self, keep=(), build_ctx: bool = False) -> int:
        """Release the context's arena buffers except those holding the device pointers in `keep`
        (g2n_context_trim) and torch's cached blocks: a sharded rank's dictionary, touch descriptors
        and partition buffers between protocol stages.  Returns the bytes the arena released."""
        ctx = self.ctx_b if build_ctx else self.ctx
        if not ctx:
            return 0
        ptrs = [int(p) for p in keep if p]
        arr = (ctypes.c_void_p * max(len(ptrs), 1))(*ptrs)
        freed = ctypes.c_uint64(0)
        self._sync()
        self._check(self.lib.g2n_context_trim(ctx, arr, len(ptrs), ctypes.byref(freed)), "g2n_context_trim")
        if self.torch is not None:
            self.torch.cuda.empty_cache()
        return int(freed.value)

    def _build_ctx(self):
        if self.ctx_b is None:
            self.ctx_b = self.lib.g2n_context_create(self.device_index)
            if not self.ctx_b:
                raise nat.NativeUnavailable(nat.last_error())
        return self.ctx_b

    def local_build(self, buf, opts: dict, unknown_warned: bool = False, view: bool = False,
                    values: bool = True) -> LocalShard:
        """The range on its own (local ids, names).  view: the COO as DevArray views of the build
        context (valid until its next build; remap_pairs rewrites them in place), the names copied.
        values=False: a build without a weight tag leaves its values unwritten (options.range_flags
        G2N_RANGE_NO_VALUES) — the caller routes coordinates only and never reads them."""
        o = nat.make_options(output=nat.OUT_COO, want_node_names=True, device=self.device_index, **opts)
        o.unknown_warned = int(unknown_warned)
        o.range_flags = 0 if values else nat.RANGE_NO_VALUES
        res = nat.Result()
        ctx = self._build_ctx() if view else self.ctx
        self._sync()
        rc = self.lib.g2n_build_device(ctx, buf.data_ptr() if buf.numel() else None, buf.numel(),
                                       ctypes.byref(o), ctypes.byref(res))
        if rc not in (0,) and not (1 <= rc <= 12):
            self._check(rc, "g2n_build_device")
        sh = LocalShard(status=rc, err_line=res.err_line, err_index=res.err_index, err_value=res.err_value,
                        err_detail=b"", warn_line=res.warn_line, has_warning=bool(res.has_warning),
                        warn_byte=res.warn_byte, n_lines=res.n_lines, n_records=res.n_records,
                        n_records_before_error=res.n_records_before_error, n_edges=res.n_edges,
                        n_local_nodes=res.n_nodes, n_cast_overflow=res.n_cast_overflow)
        for j in range(res.n_phases):
            name = res.phase_names[j].decode()
            if not name.startswith("_"):
                sh.phase_ms[name] = sh.phase_ms.get(name, 0.0) + res.phase_ms[j]
        if rc == 8 and res.err_detail_len:  # the bytes whose decode raises, for the message
            sh.err_detail = bytes(self._copy_out(res.err_detail, res.err_detail_len, "uint8").cpu().numpy())
        if rc != 0:
            return sh
        n = res.nnz
        tdt = TORCH_DTYPES[opts.get("dtype", "float64")]
        if view:
            sh.rows, sh.cols = DevArray(res.rows or 0, n, 4), DevArray(res.cols or 0, n, 4)
            sh.data = DevArray(res.data or 0, n, np.dtype(tdt).itemsize)
        else:
            sh.rows = self._copy_out(res.rows, n, "int32")
            sh.cols = self._copy_out(res.cols, n, "int32")
            sh.data = self._copy_out(res.data, n, tdt)
        sh.names_offsets = self._copy_out(res.names_offsets, res.n_nodes + 1, "int64")
        sh.names_blob = self._copy_out(res.names_blob, int(res.names_bytes), "uint8")
        return sh

    def read_range(self, path: str, offset: int, length: int):
        """Bytes [offset, offset + length) of the file, pread into pinned staging and copied to this
        rank's HBM (g2n_upload_file_range): a rank never reads the other ranks' bytes."""
        t = self._empty(length, "uint8")
        if length:
            self._sync()
            self._check(self.lib.g2n_upload_file_range(os.fsencode(path), offset, length, t.data_ptr(),
                                                       self.device_index), "g2n_upload_file_range")
        return t

    def upload(self, arr):
        """Host bytes (a numpy uint8 array: a chunk of text inflated / read into host memory) to this
        GPU's HBM."""
        t = self._empty(len(arr), "uint8")
        if len(arr):
            a = np.ascontiguousarray(arr)
            self._sync()
            if self._hip.hipMemcpy(t.data_ptr(), a.ctypes.data, len(a), 1) != 0:  # host to device
                raise RuntimeError("hipMemcpy failed")
        return t

    def free_memory(self) -> int:
        """Free HBM on this GPU (hipMemGetInfo through the C-ABI)."""
        return nat.device_memory(self.device_index)[0]

    def reset(self):
        """Release both build contexts' grow-only arenas and torch's cached blocks, keeping a fresh
        context: before a chunked build's whole-matrix assembly, whose buffers then
        have the GPU to themselves.  Views of earlier results become invalid."""
        self.close()
        if self.torch is not None:
            self.torch.cuda.empty_cache()
        self.ctx = self.lib.g2n_context_create(self.device_index)
        if not self.ctx:
            raise nat.NativeUnavailable(nat.last_error())

    def count(self, buf):
        """{lines, S lines, edge records, records} of the range (g2n_count_device: K1 only)."""
        out = (ctypes.c_int64 * 4)()
        self._sync()
        self._check(self.lib.g2n_count_device(self.ctx, buf.data_ptr() if buf.numel() else None, buf.numel(), out),
                    "g2n_count_device")
        return [int(v) for v in out]

    def build_decimal(self, buf, opts: dict, s_base: int, n_seg: int, view: bool = False, values: bool = True):
        """The range parsed straight into GLOBAL decimal ids (S lines s_base.. of n_seg), or None when
        it needs the general protocol (ids that are not decimal, errors, warnings, slow weights).
        view: the COO as DevArray views of the build context (valid until the next build_decimal)."""
        o = nat.make_options(output=nat.OUT_COO, want_node_names=False, device=self.device_index, **opts)
        o.range_s_base, o.range_n_segments = int(s_base), int(n_seg)
        o.range_flags = nat.RANGE_DECIMAL | (0 if values else nat.RANGE_NO_VALUES)
        res = nat.Result()
        self._build_ctx()
        self._sync()
        rc = self.lib.g2n_build_device(self.ctx_b, buf.data_ptr() if buf.numel() else None, buf.numel(),
                                       ctypes.byref(o), ctypes.byref(res))
        if rc != 0:
            if rc not in (nat.E_UNSUPPORTED,) and not (1 <= rc <= 12):
                self._check(rc, "g2n_build_device")
            return None
        return self._decimal_shard(res, opts, view)

    def build_decimal_range(self, buf, opts: dict, view: bool = False, values: bool = True, slots: bool = False):
        """The range parsed into GLOBAL decimal ids before the ranges' counts are known (one pass, no
        count: g2n_build_decimal_range): (LocalShard, evidence [lines, S lines, edges, records, d,
        largest edge key]) — the caller checks d against the S lines before the range and the key
        against the file's S count — or None when the one pass declines (count + build_decimal then).
        slots (view, no values): the COO may stay in the parse's group slots (LocalShard.slots), read
        only by route_slots / csr_slots."""
        o = nat.make_options(output=nat.OUT_COO, want_node_names=False, device=self.device_index, **opts)
        o.range_flags = 0 if values else nat.RANGE_NO_VALUES  # values: the caller reads them (a COO result, weights)
        if slots and view and not values:
            o.range_flags |= nat.RANGE_SLOTS
        res = nat.Result()
        ev = (ctypes.c_int64 * 6)()
        self._build_ctx()
        self._sync()
        rc = self.lib.g2n_build_decimal_range(self.ctx_b, buf.data_ptr() if buf.numel() else None, buf.numel(),
                                              ctypes.byref(o), ev, ctypes.byref(res))
        if rc != 0:
            if rc not in (nat.E_UNSUPPORTED,) and not (1 <= rc <= 12):
                self._check(rc, "g2n_build_decimal_range")
            return None
        return self._decimal_shard(res, opts, view), [int(v) for v in ev]

    def _decimal_shard(self, res, opts: dict, view: bool) -> LocalShard:
        n = res.nnz
        sh = LocalShard(status=0, err_line=-1, err_index=-1, err_value=0.0, err_detail=b"", warn_line=-1,
                        has_warning=False, warn_byte=0, n_lines=res.n_lines, n_records=res.n_records,
                        n_records_before_error=res.n_records, n_edges=res.n_edges, n_local_nodes=res.n_nodes,
                        n_cast_overflow=res.n_cast_overflow)
        tdt = TORCH_DTYPES[opts.get("dtype", "float64")]
        gc, ng, cap = ctypes.c_void_p(), ctypes.c_uint64(0), ctypes.c_uint64(0)
        if view and self.lib.g2n_context_group_slots(self.ctx_b, ctypes.byref(gc), ctypes.byref(ng),
                                                     ctypes.byref(cap)) == 0 and ng.value:
            cap_all = ng.value * cap.value  # (the slots' capacity: views over every group's slot)
            sh.rows, sh.cols = DevArray(res.rows or 0, cap_all, 4), DevArray(res.cols or 0, cap_all, 4)
            sh.data = None
            sh.slots, sh.n_trip = (gc.value, ng.value, cap.value), n
        elif view:
            sh.rows, sh.cols = DevArray(res.rows or 0, n, 4), DevArray(res.cols or 0, n, 4)
            sh.data = DevArray(res.data or 0, n, np.dtype(tdt).itemsize)
        else:
            sh.rows = self._copy_out(res.rows, n, "int32")
            sh.cols = self._copy_out(res.cols, n, "int32")
            sh.data = self._copy_out(res.data, n, tdt)
        sh.parse_path = "k1" if any(res.phase_names[k] == b"tiles" for k in range(res.n_phases)) else "tile_local"
        return sh

    def partition_keys(self, blob, offsets, n_ranks: int):
        torch = self.torch
        n = offsets.numel() - 1
        oblob = torch.empty_like(blob)
        ooffs = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        oidx = torch.empty(n, dtype=torch.int32, device=self.device)
        starts = torch.empty(n_ranks + 1, dtype=torch.int32, device=self.device)
        self._sync()
        self._check(self.lib.g2n_partition_keys(self.ctx, blob.data_ptr() if blob.numel() else None, blob.numel(),
                                                offsets.data_ptr(), n, n_ranks,
                                                oblob.data_ptr() if blob.numel() else None, ooffs.data_ptr(),
                                                oidx.data_ptr() if n else None, starts.data_ptr()),
                    "g2n_partition_keys")
        return oblob, ooffs, oidx, starts

    def dedup_keys(self, blob, offsets):
        torch = self.torch
        n = offsets.numel() - 1
        ids = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        first = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        nd = ctypes.c_uint64(0)
        self._sync()
        self._check(self.lib.g2n_dedup_keys(self.ctx, blob.data_ptr() if blob.numel() else None, blob.numel(),
                                            offsets.data_ptr(), n, ids.data_ptr(), first.data_ptr(),
                                            ctypes.byref(nd)), "g2n_dedup_keys")
        return ids[:n], first[:nd.value], nd.value

    def keyset(self):
        """A growing device set of byte keys, ids in insertion order (g2n_keyset_*)."""
        return _HipKeyset(self)

    def gather_keys(self, blob, offsets, index, nbytes: int):
        """Keys index[j] of the blob in that order: (blob of nbytes, offsets)."""
        torch = self.torch
        n = index.numel()
        oblob = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)
        ooffs = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        got = ctypes.c_uint64(0)
        self._sync()
        self._check(self.lib.g2n_gather_keys(self.ctx, blob.data_ptr() if blob.numel() else None,
                                             offsets.data_ptr(), index.data_ptr() if n else None, n,
                                             oblob.data_ptr(), nbytes, ooffs.data_ptr(), ctypes.byref(got)),
                    "g2n_gather_keys")
        return oblob[:got.value], ooffs

    def order_keys(self, first_of, src_idx, src_counts):
        """Each distinct key's order key (source rank << 32 | its local id there) — g2n_order_keys."""
        torch = self.torch
        nd = first_of.numel()
        out = torch.empty(max(nd, 1), dtype=torch.int64, device=self.device)
        ends = np.cumsum(np.asarray(src_counts, dtype=np.uint64)).astype(np.uint64)
        self._sync()
        self._check(self.lib.g2n_order_keys(self.ctx, first_of.data_ptr() if nd else None,
                                            src_idx.data_ptr() if nd else None, nd, ends.ctypes.data, len(ends),
                                            out.data_ptr()), "g2n_order_keys")
        return out[:nd]

    def rank_keys(self, keys, all_keys, rank: int):
        """Global ids: each key's index plus the smaller keys of every other owner (g2n_rank_keys)."""
        torch = self.torch
        n = keys.numel()
        out = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)
        offs = np.zeros(len(all_keys) + 1, dtype=np.uint64)
        offs[1:] = np.cumsum([x.numel() for x in all_keys])
        flat = torch.cat([x.to(self.device) for x in all_keys]) if len(all_keys) > 1 else all_keys[0]
        self._sync()
        self._check(self.lib.g2n_rank_keys(self.ctx, keys.data_ptr() if n else None, n,
                                           flat.data_ptr() if flat.numel() else None, offs.ctypes.data, len(all_keys),
                                           rank, out.data_ptr()), "g2n_rank_keys")
        return out[:n]

    def remap_pairs(self, rows, cols, gmap):
        """rows / cols (int32) through the local -> global id map, in place."""
        n = rows.numel()
        self._sync()
        self._check(self.lib.g2n_remap_pairs(self.ctx, gmap.data_ptr() if gmap.numel() else None, gmap.numel(),
                                             rows.data_ptr() if n else None, cols.data_ptr() if n else None, n),
                    "g2n_remap_pairs")
        return rows, cols

    def route_triplets(self, rows, cols, data, dtype: str, gmap, n_global: int, n_ranks: int, transposed: bool):
        n = rows.numel()
        orows = self._empty(n, "int32")
        ocols = self._empty(n, "int32")
        # data None: uniform values (unweighted), nothing to route
        odata = None if data is None else self._empty(n, TORCH_DTYPES[dtype])
        starts = self._empty(n_ranks + 1, "int32")
        self._sync()
        nz = n > 0
        self._check(self.lib.g2n_route_triplets(
            self.ctx, rows.data_ptr() if nz else None, cols.data_ptr() if nz else None,
            data.data_ptr() if nz and data is not None else None, n, nat.DTYPE_CODES[dtype],
            gmap.data_ptr() if gmap is not None and gmap.numel() else None,
            n_global, n_ranks, int(transposed), orows.data_ptr() if nz else None, ocols.data_ptr() if nz else None,
            odata.data_ptr() if nz and odata is not None else None, starts.data_ptr()), "g2n_route_triplets")
        return orows, ocols, odata, starts

    def route_slots(self, local: LocalShard, n_global: int, n_ranks: int, transposed: bool):
        """route_triplets of a group-slot COO (coordinates only): (rows, cols, None, starts)."""
        n = local.n_trip
        orows = self._empty(n, "int32")
        ocols = self._empty(n, "int32")
        starts = self._empty(n_ranks + 1, "int32")
        gc, ng, cap = local.slots
        self._sync()
        nz = n > 0
        self._check(self.lib.g2n_route_group_slots(
            self.ctx, local.rows.data_ptr() if nz else None, local.cols.data_ptr() if nz else None, gc if nz else None,
            ng, cap, n, n_global, n_ranks, int(transposed), orows.data_ptr() if nz else None,
            ocols.data_ptr() if nz else None, starts.data_ptr()), "g2n_route_group_slots")
        return orows, ocols, None, starts

    def csr_slots(self, local: LocalShard, maxsym: bool, n_rows: int, dtype: str, copy: bool = True):
        """A one-rank group's whole CSR straight from the range build's group slots
        (g2n_csr_from_group_slots), or None when the partition declines (the caller then takes the
        stream-order route)."""
        res = nat.Result()
        gc, ng, cap = local.slots
        self._sync()
        rc = self.lib.g2n_csr_from_group_slots(self.ctx, local.rows.data_ptr(), local.cols.data_ptr(), gc, ng, cap,
                                               local.n_trip, int(maxsym), n_rows, nat.DTYPE_CODES[dtype],
                                               ctypes.byref(res))
        if rc == nat.E_UNSUPPORTED:
            return None
        self._check(rc, "g2n_csr_from_group_slots")
        return self._csr_out(res, n_rows, dtype, copy)

    def _csr_out(self, res, n_rows: int, dtype: str, copy: bool):
        tdt = TORCH_DTYPES[dtype]
        if not copy:
            w = np.dtype(tdt).itemsize
            iw = 8 if res.index_width == 8 else 4
            return (DevArray(res.indptr or 0, n_rows + 1, iw), DevArray(res.indices or 0, res.nnz, iw),
                    DevArray(res.data or 0, res.nnz, w))
        idx = "int64" if res.index_width == 8 else "int32"
        return (self._copy_out(res.indptr, n_rows + 1, idx), self._copy_out(res.indices, res.nnz, idx),
                self._copy_out(res.data, res.nnz, tdt))

    def csr_pair(self, a, t, maxsym: bool, row_base: int, n_rows: int, n_cols: int, dtype: str, uniform: bool,
                 force_unsorted: int, copy: bool = True):
        """The slice's CSR; copy=False: DevArray views of the context's result (valid until its next
        call — what a caller that reads the slice right away, or never, needs: no device copy)."""
        res = nat.Result()
        t = t if t is not None else (a[0][:0], a[1][:0], None)

        def p(x):  # uniform builds pass no values (None)
            return x.data_ptr() if x is not None and x.numel() else None

        self._sync()
        self._check(self.lib.g2n_csr_from_coo_pair(self.ctx, p(a[0]), p(a[1]), p(a[2]), a[0].numel(), p(t[0]),
                                                   p(t[1]), p(t[2]), t[0].numel(), int(maxsym), row_base, n_rows,
                                                   n_cols, nat.DTYPE_CODES[dtype], int(uniform), force_unsorted,
                                                   ctypes.byref(res)), "g2n_csr_from_coo_pair")
        tdt = TORCH_DTYPES[dtype]
        if not copy:
            w = np.dtype(tdt).itemsize
            iw = 8 if res.index_width == 8 else 4  # (a whole matrix past 2^31 - 1 entries: int64 views)
            return (DevArray(res.indptr or 0, n_rows + 1, iw), DevArray(res.indices or 0, res.nnz, iw),
                    DevArray(res.data or 0, res.nnz, w), not res.sum_sorted, bool(maxsym) and not res.sum_t_sorted)
        idx = "int64" if res.index_width == 8 else "int32"  # (a whole matrix past 2^31 - 1 entries)
        indptr = self._copy_out(res.indptr, n_rows + 1, idx)
        indices = self._copy_out(res.indices, res.nnz, idx)
        vals = self._copy_out(res.data, res.nnz, tdt)
        return indptr, indices, vals, not res.sum_sorted, bool(maxsym) and not res.sum_t_sorted


# ---------------------------------------------------------------------- protocol --
class Comm:
    """The collectives the protocol needs, on tensors of any device: with gloo they go through
    host memory, with nccl (RCCL over xGMI) they stay on the GPU."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.group = torch, dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.host = dist.get_backend(group) == "gloo"
        self.sent = 0  # bytes the all-to-all-v calls sent to other ranks (ShardResult.a2a_bytes_sent)

    def _c(self, x):
        return x.cpu() if self.host and x.is_cuda else x

    def a2av(self, x, send_counts):
        """all-to-all-v: send_counts[k] elements of x to rank k; returns (received, counts)."""
        outs, recv = self.a2av_multi([x], send_counts)
        return outs[0], recv

    def a2av_multi(self, xs, send_counts):
        """a2av of several tensors with the same per-rank counts: one count exchange for all of
        them (None entries pass through as None)."""
        torch = self.torch
        if self.world == 1:  # a copy, as the send-to-self part of a real all-to-all (force_protocol times it)
            return [None if x is None else x.clone() for x in xs], list(send_counts)
        ref = next(x for x in xs if x is not None)
        dev = ref.device
        host = self._c(ref[:0]).device
        sc = torch.tensor(list(send_counts), dtype=torch.int64, device=host)
        rc = torch.empty(self.world, dtype=torch.int64, device=host)
        self.dist.all_to_all_single(rc, sc, group=self.group)
        recv = [int(v) for v in rc.tolist()]
        outs = []
        for x in xs:
            if x is None:
                outs.append(None)
                continue
            xc = self._c(x.contiguous())
            self.sent += (sum(send_counts) - send_counts[self.rank]) * xc.element_size()
            out = torch.empty(sum(recv), dtype=xc.dtype, device=xc.device)
            self.dist.all_to_all_single(out, xc, output_split_sizes=recv, input_split_sizes=list(send_counts),
                                        group=self.group)
            outs.append(out.to(dev))
        return outs, recv

    def allgather_v(self, x):
        """every rank's (variable-length, 1-D) tensor, in rank order: one padded all-gather when
        the lengths are balanced (world x the longest within twice their sum — the owners' hashed
        key sets), else one broadcast per rank (no padding)"""
        torch = self.torch
        if self.world == 1:
            return [x]
        xc = self._c(x.contiguous())
        n = torch.tensor([xc.numel()], dtype=torch.int64, device=xc.device)
        ns = [torch.empty_like(n) for _ in range(self.world)]
        self.dist.all_gather(ns, n, group=self.group)
        sizes = [int(v.item()) for v in ns]
        m = max(sizes)
        if m == 0 or m * self.world > 2 * sum(sizes):
            return [t for _, t in self.parts(x, root=None, sizes=sizes)]
        pad = torch.zeros(m, dtype=xc.dtype, device=xc.device)
        pad[:xc.numel()] = xc
        outs = [torch.empty_like(pad) for _ in range(self.world)]
        self.dist.all_gather(outs, pad, group=self.group)
        return [o[:k].to(x.device) for o, k in zip(outs, sizes)]

    def parts(self, x, root=None, sizes=None):
        """Yield (rank, tensor) for every rank's (variable-length, 1-D) tensor in rank order — on
        every rank (root None: one broadcast per rank) or on `root` only (point-to-point sends; the
        other ranks send theirs and yield nothing).  Tensors come back on x's device."""
        torch = self.torch
        if self.world == 1:
            yield 0, x
            return
        dev = x.device
        xc = self._c(x.contiguous())
        if sizes is None:
            n = torch.tensor([xc.numel()], dtype=torch.int64, device=xc.device)
            ns = [torch.empty_like(n) for _ in range(self.world)]
            self.dist.all_gather(ns, n, group=self.group)
            sizes = [int(v.item()) for v in ns]
        if root is not None and self.rank != root:
            if sizes[self.rank]:
                self.dist.send(xc, dst=self._global(root), group=self.group)
            return
        for k in range(self.world):
            mine = k == self.rank
            buf = xc if mine else torch.empty(sizes[k], dtype=xc.dtype, device=xc.device)
            if sizes[k]:
                if root is None:
                    self.dist.broadcast(buf, src=self._global(k), group=self.group)
                elif not mine:
                    self.dist.recv(buf, src=self._global(k), group=self.group)
            yield k, (x if mine else buf.to(dev))

    def _global(self, k):
        return k if self.group is None else self.dist.get_global_rank(self.group, k)

    def allgather_list(self, vals):
        """every rank's list of numbers (float64-exact up to 2^53)"""
        torch = self.torch
        if self.world == 1:
            return [list(vals)]
        t = torch.tensor(vals, dtype=torch.float64)
        if not self.host:
            t = t.cuda()
        outs = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(outs, t, group=self.group)
        return [[int(v) if float(v).is_integer() else v for v in o.tolist()] for o in outs]

    def bcast(self, x, src):
        if self.world == 1:
            return x
        dev = x.device
        xc = self._c(x)
        self.dist.broadcast(xc, src=src, group=self.group)
        return xc.to(dev)

    def allreduce_sum(self, vals, device):
        """element-wise sum over the ranks of a short list of ints"""
        torch = self.torch
        t = torch.tensor([int(v) for v in vals], dtype=torch.int64, device=device)
        if self.world > 1:
            tc = self._c(t)
            self.dist.all_reduce(tc, group=self.group)
            t = tc
        return [int(v) for v in t.tolist()]

    def allreduce_max(self, x):
        if self.world == 1:
            return x
        dev = x.device
        xc = self._c(x)
        self.dist.all_reduce(xc, op=self.dist.ReduceOp.MAX, group=self.group)
        return xc.to(dev)

    def allreduce_min(self, x):
        if self.world == 1:
            return x
        dev = x.device
        xc = self._c(x)
        self.dist.all_reduce(xc, op=self.dist.ReduceOp.MIN, group=self.group)
        return xc.to(dev)


def _slice(engine, C, a, tstream, maxsym, n_global, dtype, weight_tag, tm, copy_out=True):
    """Step 6: this rank's CSR row slice (rows [row_lo, row_hi) of n_global)."""
    import time

    import torch

    world, rank = C.world, C.rank
    t4 = time.perf_counter()
    row_lo = (rank * n_global + world - 1) // world
    row_hi = ((rank + 1) * n_global + world - 1) // world
    uniform = not weight_tag
    force = -1
    if not uniform and dtype in ("float32", "float64") and world > 1:
        # scipy's has_sorted_indices is a property of the whole matrix: OR over the slices
        _, _, _, ua, ut = engine.csr_pair(a, tstream, maxsym, row_lo, row_hi - row_lo, n_global, dtype, uniform, -1)
        flags = C.allreduce_max(torch.tensor([int(ua), int(ut)], dtype=torch.int64, device=engine.device))
        force = int(flags[0].item()) | (int(flags[1].item()) << 1)
    kw = {} if copy_out else {"copy": False}  # (engines without views always copy)
    indptr, indices, vals, _, _ = engine.csr_pair(a, tstream, maxsym, row_lo, row_hi - row_lo, n_global, dtype,
                                                  uniform, force, **kw)
    tm["csr"] = (time.perf_counter() - t4) * 1e3
    return row_lo, row_hi, indptr, indices, vals


def _route(engine, C, local, dtype, gmap, n_global, maxsym, uniform, tm):
    """Step 5: triplets to the owners of their rows (and the A.T stream for MAX-SYM).  Uniform
    (unweighted) values are not routed; one rank with global ids routes nothing."""
    import time

    t3 = time.perf_counter()
    if C.world == 1 and gmap is None:  # every row is this rank's: the streams as they are
        d = None if uniform else local.data
        tm["route"] = 0.0
        return (local.rows, local.cols, d), ((local.cols, local.rows, d) if maxsym else None)

    def route(transposed):
        if local.slots is not None:  # group slots (G2N_RANGE_SLOTS, uniform): the route compacts them
            rr, cc, dd, st = engine.route_slots(local, n_global, C.world, transposed)
        else:
            rr, cc, dd, st = engine.route_triplets(local.rows, local.cols, None if uniform else local.data,
                                                   local.dtype_name, gmap, n_global, C.world, transposed)
        st_l = [int(v) for v in st.tolist()]
        cnt = [st_l[k + 1] - st_l[k] for k in range(C.world)]
        return tuple(C.a2av_multi([rr, cc, dd], cnt)[0])

    a = route(False)
    tstream = route(True) if maxsym else None
    tm["route"] = (time.perf_counter() - t3) * 1e3
    return a, tstream


def _build_decimal_sharded(buf, engine, C, opts, gd, maxsym, gather_names, tm, keep_coo=False, names_root=None,
                           copy_out=True):
    """The decimal-id fast path (module docstring), or None when a range breaks its premise."""
    import time

    import torch

    world, rank = C.world, C.rank
    t0 = time.perf_counter()
    tps = 2 if opts.get("bidirected") else 1

    def premise(allc):  # no edge line may precede an S line (ids = S order); the file's S count
        seen_edge, ok = False, True
        for k in range(world):
            if allc[k][1] and seen_edge:
                ok = False
            seen_edge = seen_edge or allc[k][2] > 0
        n = int(sum(c[1] for c in allc))
        return ok and 0 < n and n * tps < 2**31 - 1, n

    local, allc = None, None
    # the COO left in the parse's group slots when nothing reads it in stream order (no COO result, unit
    # values): routed straight from them, or at one rank turned into the CSR straight from them
    slots = getattr(engine, "supports_slots", False) and not keep_coo
    if (hasattr(engine, "build_decimal_range") and not opts.get("bidirected") and not opts.get("weight_tag")
            and not opts.get("strip_orientation")):
        # one pass, no count: every range parses into global ids first and reports its evidence; one
        # all-gather decides for every rank at once (g2n_build_decimal_range)
        got = engine.build_decimal_range(buf, opts, view=not keep_coo, values=keep_coo,
                                         **({"slots": True} if slots else {}))
        alle = C.allgather_list(got[1] if got is not None else [-1] * 6)
        tm["count"] = 0.0
        if all(e[0] >= 0 for e in alle):
            allc = [e[:4] for e in alle]
            ok, n_seg = premise(allc)
            s_bases = np.cumsum([0] + [c[1] for c in allc])
            ok = ok and all(e[1] == 0 or e[4] == s_bases[k] for k, e in enumerate(alle)) and \
                max(e[5] for e in alle) <= n_seg
            if not ok:
                return None
            local = got[0]
            tm["build"] = (time.perf_counter() - t0) * 1e3
        elif all(e[0] < 0 for e in alle):
            # every range declined: names that are not the decimal ids (a shape the one pass refuses in
            # every range would be unusual) — the general protocol, without a count + build that would
            # decline again (C5 with hashed names: 5 ms per build)
            return None
        # else some range declined the one pass: count and build with the range offsets known
    if local is None:
        t0 = time.perf_counter()
        cnt = engine.count(buf)  # [lines, S lines, edges, records]
        allc = C.allgather_list(cnt)
        ok, n_seg = premise(allc)
        if not ok:
            return None
        s_base = int(sum(allc[k][1] for k in range(rank)))
        tm["count"] = (time.perf_counter() - t0) * 1e3
        local = engine.build_decimal(buf, opts, s_base, n_seg, view=not keep_coo,
                                     values=keep_coo or bool(opts.get("weight_tag")))
        # every range's ids are global decimals (the id map needs no exchange) — or nobody's are
        verdict = torch.tensor([0 if local is None else 1], dtype=torch.int64, device=engine.device)
        if int(C.allreduce_min(verdict).item()) == 0:
            return None
        tm["build"] = (time.perf_counter() - t0) * 1e3 - tm["count"]
    n_global = n_seg * tps
    local.dtype_name = opts.get("dtype", "float64")
    n_trip = local.triplets()
    got_csr = None
    if C.world == 1 and local.slots is not None:
        # one rank: no route, and the slice is the whole matrix — the single-GPU partition reads the slots
        t4 = time.perf_counter()
        tm["route"] = 0.0
        got_csr = engine.csr_slots(local, maxsym, n_global, local.dtype_name, copy=copy_out)
        if got_csr is None:  # the partition declined (an overfull bucket): the range's stream-order COO
            again = engine.build_decimal_range(buf, opts, view=True, values=False)
            if again is None:  # (one rank: the general protocol decides alone)
                return None
            local = again[0]
            local.dtype_name = opts.get("dtype", "float64")
        else:
            tm["csr"] = (time.perf_counter() - t4) * 1e3
            row_lo, row_hi = 0, n_global
            indptr, indices, vals = got_csr
    if got_csr is None:
        a, tstream = _route(engine, C, local, local.dtype_name, None, n_global, maxsym, not opts.get("weight_tag"),
                            tm)
        row_lo, row_hi, indptr, indices, vals = _slice(engine, C, a, tstream, maxsym, n_global, local.dtype_name,
                                                       opts.get("weight_tag"), tm, copy_out)
    sums = C.allreduce_sum([local.n_cast_overflow, int(indices.numel()), n_trip], engine.device)
    out = ShardResult(status=0, n_lines=int(sum(c[0] for c in allc)), n_records=int(sum(c[3] for c in allc)),
                      n_edges=int(sum(c[2] for c in allc)), n_nodes=n_global, row_lo=row_lo, row_hi=row_hi,
                      indptr=indptr, indices=indices, data=vals, n_cast_overflow=sums[0],
                      index_maxval=sums[1] if maxsym else sums[2])
    out.n_records_before_error = out.n_records
    if gather_names and names_root in (None, rank):  # node k is str(k + 1) (bidirected: k // 2 + 1 and ":+" / ":-")
        out.names_blob, out.names_offsets = nat.decimal_names(n_global, bool(opts.get("bidirected")))
    out.timings_ms = tm
    out.a2a_bytes_sent = C.sent
    out.fast_path = True
    out.parse_path = getattr(local, "parse_path", "")
    out.coo_layout = "group_slots" if getattr(local, "slots", None) is not None else "stream"
    if keep_coo:
        out.coo = (local.rows, local.cols, local.data)
    return out


class FileSource:
    """A plain file on disk: each chunk is pread straight into HBM (g2n_upload_file_range)."""

    def __init__(self, path):
        self.path = str(path)
        self.size = os.path.getsize(self.path)

    def ranges(self, n: int):
        return file_line_ranges(self.path, n)

    def upload(self, engine, lo: int, hi: int):
        return engine.read_range(self.path, lo, hi - lo)


class HostSource:
    """Bytes already in host memory — a ``.gz`` inflated on the host, stdin, a file object's read():
    each chunk is copied to HBM on its own."""

    def __init__(self, data):
        self.arr = data if isinstance(data, np.ndarray) else np.frombuffer(data, dtype=np.uint8)
        self.size = len(self.arr)

    def ranges(self, n: int):
        return line_ranges(self.arr, n)

    def upload(self, engine, lo: int, hi: int):
        return engine.upload(self.arr[lo:hi])


def _as_source(src):
    return src if hasattr(src, "ranges") else FileSource(src)


_ITEMSIZE = {"bool": 1, "int8": 1, "int32": 4, "float32": 4, "float64": 8}


def csr_bytes_estimate(n_a: int, n_t: int, n_rows: int, w: int) -> int:
    """HBM one g2n_csr_from_coo_pair call over n_a A entries and n_t A.T entries takes beyond its
    inputs — the bucket partition's two element buffers and pair words, the staged merged entries,
    the result (int32 or int64 indices, w-byte values) and the count matrices — an upper bound
    (g2n_pipeline.hip csr_partition / csr_partition_w)."""
    n_el = n_a + n_t
    return int(n_el * (40 + w) + 24 * n_rows + (256 << 20))


class ChunkedAssemblyTooLarge(MemoryError):
    pass


def _np(x):
    return x if isinstance(x, np.ndarray) else x.cpu().numpy()


def _assemble_csr(engine, parts, n: int, maxsym: bool, uniform: bool, dtype: str, tm: dict, free_hbm, bands=None):
    """The whole matrix's CSR over every chunk's triplets (parts: per chunk (rows, cols, data) device
    tensors, stream order): one g2n_csr_from_coo_pair when it fits the GPU's free HBM, else in row
    bands — each chunk's triplets routed by band (g2n_route_triplets: stable, so every row keeps its
    stream order and scipy's duplicate-summation order), each band's CSR built (row_base) and copied
    to host memory, the bands' indptrs rebased (the sharded gather's rule, concat_indptr).  Returns
    (indptr, indices, data, index_maxval) — device tensors (one piece) or numpy (bands)."""
    import time

    t1 = time.perf_counter()
    n_trip = sum(int(p[0].numel()) for p in parts)
    w = _ITEMSIZE[dtype]
    wv = 0 if uniform else w
    engine.reset()  # the chunk builds' arenas go before the assembly's buffers come
    free = int(free_hbm())
    n_t = n_trip if maxsym else 0
    whole = csr_bytes_estimate(n_trip, n_t, n, w) + n_trip * (8 + wv) * (2 if maxsym else 1)
    if bands is None:
        bands = 1 if whole <= free else None
    if bands is None:
        routed = n_trip * (8 + wv) * (2 if maxsym else 1)  # the band-ordered copies (A, and A.T for MAX-SYM)
        room = free - routed - n_trip * (8 + wv)  # the chunks' own triplets while they are routed
        per = csr_bytes_estimate(n_trip, n_t, n, w)
        if room <= per // 64:
            raise ChunkedAssemblyTooLarge(
                f"parse_gfa: the CSR of {n_trip} triplets over {n} nodes needs about {(whole + routed) / 1e9:.1f} GB "
                f"of HBM even in row bands; {free / 1e9:.1f} GB free")
        bands = max(2, -(-per // int(room * 0.8)))
    d = lambda x: None if uniform else x  # noqa: E731  (uniform values are never read)
    if bands == 1:
        cat = engine.cat
        rows, cols = cat([p[0] for p in parts]), cat([p[1] for p in parts])
        data = None if uniform else cat([p[2] for p in parts])
        parts.clear()
        indptr, indices, vals, _, _ = engine.csr_pair((rows, cols, data), (cols, rows, data) if maxsym else None, maxsym,
                                                      0, n, n, dtype, uniform, -1)
        tm["csr"] = (time.perf_counter() - t1) * 1e3
        return indptr, indices, vals, int(indices.numel()) if maxsym else n_trip
    # row bands: rank k of a `bands`-rank sharded build owns rows [ceil(k n / B), ceil((k+1) n / B))
    ra, rt = [], []
    while parts:
        r, c, x = parts.pop(0)
        ra.append(engine.route_triplets(r, c, d(x), dtype, None, n, bands, False))
        if maxsym:
            rt.append(engine.route_triplets(r, c, d(x), dtype, None, n, bands, True))
        del r, c, x
    starts_a = [[int(v) for v in s[3].tolist()] for s in ra]
    starts_t = [[int(v) for v in s[3].tolist()] for s in rt]

    def band(routed, starts, k):
        pieces = [(g[0][s[k]:s[k + 1]], g[1][s[k]:s[k + 1]], None if g[2] is None else g[2][s[k]:s[k + 1]])
                  for g, s in zip(routed, starts)]
        cat = engine.cat
        return (cat([p[0] for p in pieces]), cat([p[1] for p in pieces]),
                None if uniform else cat([p[2] for p in pieces]))

    force = -1
    if not uniform and dtype in ("float32", "float64"):
        # scipy's has_sorted_indices is a property of the whole matrix: OR over the bands first
        fa = ft = 0
        for k in range(bands):
            lo, hi = (k * n + bands - 1) // bands, ((k + 1) * n + bands - 1) // bands
            _, _, _, ua, ut = engine.csr_pair(band(ra, starts_a, k), band(rt, starts_t, k) if maxsym else None,
                                              maxsym, lo, hi - lo, n, dtype, uniform, -1)
            fa, ft = fa | int(ua), ft | int(ut)
        force = fa | (ft << 1)
    ptrs, idx, vals = [], [], []
    for k in range(bands):
        lo, hi = (k * n + bands - 1) // bands, ((k + 1) * n + bands - 1) // bands
        ip, ix, vv, _, _ = engine.csr_pair(band(ra, starts_a, k), band(rt, starts_t, k) if maxsym else None, maxsym,
                                           lo, hi - lo, n, dtype, uniform, force)
        ptrs.append(_np(ip).astype(np.int64))
        idx.append(_np(ix))
        vals.append(_np(vv))
        del ip, ix, vv
    ra.clear()
    rt.clear()
    nnz = sum(len(x) for x in idx)
    idt = scipy_index_dtype(nnz if maxsym else n_trip, n)
    indptr = concat_indptr(ptrs, idt)
    indices = np.concatenate(idx).astype(idt, copy=False) if idx else np.zeros(0, dtype=idt)
    data = np.concatenate(vals) if vals else np.zeros(0)
    tm["csr"] = (time.perf_counter() - t1) * 1e3
    tm["csr_bands"] = bands
    return indptr, indices, data, nnz if maxsym else n_trip


def build_chunked(source, *, engine, chunk_bytes: int, directed=True, bidirected=False, keep_directed_bidir=False,
                  asymmetric=False, strip_orientation=False, dtype="float64", weight_tag=None, gather_names=False,
                  keep_coo=False, free_hbm=None, bands=None) -> ShardResult | None:
    """One file whose working set does not fit one GPU, built on that GPU alone in line-aligned chunks
    of about `chunk_bytes`: the decimal-id chunks (`_chunked_decimal`) when the file's names are
    "1".."N" in S-first order and the build is plain, else chunks with local ids merged into one
    dictionary as they come (`_chunked_general`).  `source`: a path (FileSource) or a HostSource.
    Parse errors, cast errors and the one-shot unsupported-record warning are resolved across the
    chunks in stream order, as one piece would raise / emit them (build_sharded's rule).  The
    whole-matrix CSR is assembled after the chunk builds' arenas are released, in row bands when it
    does not fit (`_assemble_csr`); a COO result (keep_coo without MAX-SYM) is kept in host memory
    chunk by chunk.  None only past 2^31 - 1 nodes (the one-piece build reports that limit)."""
    src = _as_source(source)
    free_hbm = free_hbm or engine.free_memory
    kw = dict(engine=engine, chunk_bytes=chunk_bytes, directed=directed, keep_directed_bidir=keep_directed_bidir,
              asymmetric=asymmetric, dtype=dtype, gather_names=gather_names, keep_coo=keep_coo, free_hbm=free_hbm,
              bands=bands)
    if not (bidirected or weight_tag or strip_orientation):
        got = _chunked_decimal(src, **kw)
        if got is not None:
            return got
    return _chunked_general(src, bidirected=bidirected, strip_orientation=strip_orientation, weight_tag=weight_tag,
                            **kw)


def _keep_part(keep_host: bool, rows, cols, data):
    """A chunk's stream-order triplets, kept on the device (the CSR is built over them) or moved to
    host memory (a COO result never needs them on the GPU again)."""
    if keep_host:
        return _np(rows).copy(), _np(cols).copy(), _np(data).copy()
    return rows, cols, data


def _finish_chunked(engine, out, parts, n, maxsym, uniform, dtype, keep_coo, tm, free_hbm, bands):
    out.row_lo, out.row_hi = 0, n
    if keep_coo and not maxsym:  # parse_gfa's stream-order COO, already in host memory
        out.coo = tuple(np.concatenate([p[j] for p in parts]) if parts else np.zeros(0, np.int32) for j in range(3))
        out.index_maxval = int(len(out.coo[0]))
        return out
    if keep_coo:
        out.coo = tuple(np.concatenate([_np(p[j]) for p in parts]) for j in range(3))
    out.indptr, out.indices, out.data, out.index_maxval = _assemble_csr(engine, parts, n, maxsym, uniform, dtype, tm,
                                                                        free_hbm, bands)
    return out


def _chunked_general(src, *, engine, chunk_bytes: int, directed, bidirected, keep_directed_bidir, asymmetric,
                     strip_orientation, dtype, weight_tag, gather_names, keep_coo, free_hbm=None,
                     bands=None) -> ShardResult | None:
    """Chunks in stream order, any names: each chunk is built on its own (local first-touch ids, its
    distinct keys in local id order), then its keys are deduplicated together with the file's keys
    so far, those first (`dedup_keys` keeps arrival order: a known key gets its global id, a new one
    the next id in the chunk's first-touch order — which is the file's, since every earlier chunk
    came first), the new keys appended to the file's names (`gather_keys`) and the chunk's triplets
    remapped to global ids (`remap_pairs`).  The CSR / COO is built once over all chunks' triplets.
    Stream-order resolution (parser.py:114-132, builders.py:281): the first parse error ends the
    build with its global line; a cast error is kept while later chunks are parsed (a later parse
    error still wins, as the reference casts after its loop); the first unsupported record warns once
    and every later chunk is built with it already warned (options.unknown_warned)."""
    import time

    src = _as_source(src)
    free_hbm = free_hbm or engine.free_memory
    opts = dict(directed=directed, bidirected=bidirected, keep_directed_bidir=keep_directed_bidir,
                asymmetric=asymmetric, strip_orientation=strip_orientation, dtype=dtype, weight_tag=weight_tag)
    gd = keep_directed_bidir or (not bidirected and directed)  # builders.py:143
    maxsym = gd and not asymmetric                               # builders.py:282
    uniform = not weight_tag
    keep_host = keep_coo and not maxsym
    n_chunks = max(1, -(-src.size // max(1, int(chunk_bytes))))
    t0 = time.perf_counter()
    dev = engine.device
    ks = engine.keyset()  # the file's distinct keys so far, in global id order
    n_g = 0
    parts = []
    n_lines = n_records = n_edges = overflow = n_trip = 0
    warned = None      # (global warn line, warn byte) of the first unsupported record
    cast_err = None    # (status, global triplet index, value) of the first cast error
    tm = {"read": 0.0, "local_build": 0.0, "merge_keys": 0.0, "remap": 0.0}

    def lap(key, t):
        tm[key] += (time.perf_counter() - t) * 1e3
        return time.perf_counter()

    def result(**kw):
        r = ShardResult(n_lines=n_lines, n_records=n_records, n_edges=n_edges, n_nodes=n_g,
                        n_cast_overflow=overflow, **kw)
        if warned is not None:
            r.has_warning, r.warn_line, r.warn_byte = True, warned[0], warned[1]
        return r

    try:
        for lo, hi in src.ranges(n_chunks):
            t = time.perf_counter()
            buf = src.upload(engine, lo, hi)
            t = lap("read", t)
            sh = engine.local_build(buf, opts, unknown_warned=warned is not None)
            if warned is None and sh.has_warning and not (sh.status == 8 and sh.err_line == sh.warn_line):
                warned = (n_lines + sh.warn_line, sh.warn_byte)
            del buf
            t = lap("local_build", t)
            if sh.status != 0 and sh.status not in CAST_ERRORS:  # a parse error: the build ends here
                if warned is not None and warned[0] >= n_lines + sh.err_line:
                    warned = None  # (the warning would have come after the error)
                out = result(status=int(sh.status), err_line=n_lines + int(sh.err_line), err_detail=sh.err_detail)
                out.n_lines, out.n_records = n_lines + int(sh.n_lines), n_records + int(sh.n_records)
                out.n_records_before_error = n_records + int(sh.n_records_before_error)
                return out
            n_lines += int(sh.n_lines)
            n_records += int(sh.n_records)
            if sh.status in CAST_ERRORS:
                if cast_err is None:
                    cast_err = (int(sh.status), n_trip + int(sh.err_index), float(sh.err_value))
                continue
            n_edges += int(sh.n_edges)
            overflow += int(sh.n_cast_overflow)
            if cast_err is not None:
                continue  # (the build raises the cast error; only later parse errors still matter)
            n_l = int(sh.n_local_nodes)
            ids, n_g = ks.add(sh.names_blob.to(dev), sh.names_offsets.to(dev))
            t = lap("merge_keys", t)
            rows, cols = sh.rows, sh.cols
            if n_l and rows.numel():
                rows, cols = engine.remap_pairs(rows, cols, ids[:n_l].contiguous())
            t = lap("remap", t)
            n_trip += int(rows.numel())
            parts.append(_keep_part(keep_host, rows, cols, sh.data))
            del rows, cols, sh
        if cast_err is not None:
            return result(status=cast_err[0], err_index=cast_err[1], err_value=cast_err[2])
        n = n_g
        if n >= INT32_MAX:
            return None
        tm["build"] = (time.perf_counter() - t0) * 1e3
        out = result(status=0)
        out.n_records_before_error = n_records
        if gather_names:
            nb, no = ks.names()
            out.names_blob, out.names_offsets = nb.cpu().numpy(), no.cpu().numpy()
        ks.close()  # before the assembly: its memory goes, and the engine's reset replaces the context
        _finish_chunked(engine, out, parts, n, maxsym, uniform, dtype, keep_coo, tm, free_hbm, bands)
        out.parse_path = "chunked general"
        out.timings_ms = tm
        return out
    finally:
        ks.close()


def _chunked_decimal(src, *, engine, chunk_bytes: int, directed=True, keep_directed_bidir=False, asymmetric=False,
                     dtype="float64", gather_names=False, keep_coo=False, free_hbm=None,
                     bands=None) -> ShardResult | None:
    """One file whose working set does not fit one GPU, on that GPU alone: its line-aligned byte
    ranges of about `chunk_bytes` are uploaded and parsed one after another straight into GLOBAL
    decimal ids — the sharded fast path's one pass (`build_decimal_range`) — so only one range's text
    and working set are resident at a time beside the growing COO.  Each range's premise evidence
    is checked as it comes (the rule of `_build_decimal_sharded`: S lines first, each range's names
    continuing the S lines before it), every edge key against the S count at the end; the CSR (or,
    keep_coo, the stream-order COO) is then built once over all ranges' triplets.  Returns the whole
    matrix as one row slice, or None when the decimal-id premise fails anywhere (names not "1".."N"
    in S-first order, an error or warning in a range): the caller then runs the merged-dictionary
    chunks, which resolve errors and warnings in stream order."""
    import time

    src = _as_source(src)
    free_hbm = free_hbm or engine.free_memory
    opts = dict(directed=directed, bidirected=False, keep_directed_bidir=keep_directed_bidir, asymmetric=asymmetric,
                strip_orientation=False, dtype=dtype, weight_tag=None)
    gd = keep_directed_bidir or directed  # builders.py:143 (not bidirected)
    maxsym = gd and not asymmetric        # builders.py:282
    keep_host = keep_coo and not maxsym
    n_chunks = max(1, -(-src.size // max(1, int(chunk_bytes))))
    tm = {}
    t0 = time.perf_counter()
    parts, ev = [], []
    overflow = 0
    seen_edge, s_before, vmax = False, 0, 0
    for lo, hi in src.ranges(n_chunks):
        buf = src.upload(engine, lo, hi)
        got = engine.build_decimal_range(buf, opts, view=False, values=keep_coo)
        del buf
        if got is None:
            return None
        sh, e = got
        e = [int(v) for v in e]  # [lines, S lines, edges, records, d, largest edge key]
        if e[1] and (seen_edge or e[4] != s_before):
            return None  # an S line after an edge line, or names not continuing the S lines before
        seen_edge = seen_edge or e[2] > 0
        s_before += e[1]
        vmax = max(vmax, e[5])
        parts.append(_keep_part(keep_host, sh.rows, sh.cols, sh.data))
        overflow += int(sh.n_cast_overflow)
        ev.append(e)
        del sh
    n = s_before
    if not 0 < n < INT32_MAX or vmax > n:
        return None
    tm["build"] = (time.perf_counter() - t0) * 1e3
    out = ShardResult(status=0, n_lines=sum(e[0] for e in ev), n_records=sum(e[3] for e in ev),
                      n_edges=sum(e[2] for e in ev), n_nodes=n, n_cast_overflow=overflow)
    out.n_records_before_error = out.n_records
    if gather_names:  # node k is str(k + 1)
        out.names_blob, out.names_offsets = nat.decimal_names(n, False)
    _finish_chunked(engine, out, parts, n, maxsym, True, dtype, keep_coo, tm, free_hbm, bands)
    out.fast_path = True
    out.parse_path = f"chunked x{len(ev)}"
    out.timings_ms = tm
    return out


def build_sharded(buf, *, engine, group=None, directed=True, bidirected=False, keep_directed_bidir=False,
                  asymmetric=False, strip_orientation=False, dtype="float64", weight_tag=None,
                  gather_names=False, keep_coo=False, names_root=None, force_protocol=False,
                  copy_out=True, trim=False) -> ShardResult:
    """Build this rank's byte range `buf` (uint8 tensor on the engine's device) as part of one
    file split over `group` in rank order; returns this rank's CSR row slice (and, keep_coo, the
    range's stream-order triplets over global ids: res.coo = (rows, cols, data)).
    gather_names: the node names in id order (res.names_blob / names_offsets) on every rank, or
    on rank `names_root` only.  force_protocol: run the general exchange even on one rank (whose
    local ids are the global ones; measurement of the protocol's cost only).  copy_out=False: the slice's
    indptr / indices / data are views of the engine's context (no device copy; valid until the engine's
    next call) — the bench's timed steps, which never read them.  trim: release each context's dead
    buffers between the general protocol's stages (engine.trim: the local dictionary once the range's
    COO and names are out, the owners' dedup table once the global ids are known) — the HBM of a
    rank that shares its GPU, at the cost of re-allocating them on the next build."""
    import time

    import torch
    import torch.distributed as dist

    C = Comm(group)
    world, rank = C.world, C.rank
    dev = engine.device
    opts = dict(directed=directed, bidirected=bidirected, keep_directed_bidir=keep_directed_bidir,
                asymmetric=asymmetric, strip_orientation=strip_orientation, dtype=dtype, weight_tag=weight_tag)
    gd = keep_directed_bidir or (not bidirected and directed)  # builders.py:143
    maxsym = gd and not asymmetric                               # builders.py:282
    tpe = 4 if (bidirected and not keep_directed_bidir) else 2
    ktrip = 4 if tpe == 4 else (1 if gd else 2)
    tm = {}
    fast = None if force_protocol else _build_decimal_sharded(buf, engine, C, opts, gd, maxsym, gather_names, tm,
                                                               keep_coo, names_root, copy_out)
    if fast is not None:
        return fast
    t0 = time.perf_counter()

    # 1. local build; 2. stream-order resolution of errors and the one-shot warning
    view = not keep_coo and getattr(engine, "supports_views", False)
    # (uniform values are never routed: a view build, whose COO nobody else reads, skips writing them)
    local = engine.local_build(buf, opts, view=True, values=bool(weight_tag)) if view else engine.local_build(buf, opts)

    def stats(sh):
        return [sh.status, sh.err_line, sh.warn_line, sh.n_lines, sh.n_records, sh.n_records_before_error,
                sh.n_edges, sh.n_cast_overflow]

    allst = C.allgather_list(stats(local))
    first_unk = next((k for k in range(world) if allst[k][2] >= 0), None)
    if first_unk is not None and rank > first_unk and local.warn_line >= 0:
        # an earlier range already warned: this range's unsupported records are silent
        if local.status == 8 and local.err_line == local.warn_line:
            local = (engine.local_build(buf, opts, unknown_warned=True, view=True, values=bool(weight_tag)) if view
                     else engine.local_build(buf, opts, unknown_warned=True))
        local.has_warning = False
    if first_unk is not None:  # a range may have been rebuilt: its counts again
        allst = C.allgather_list(stats(local))
    if trim and view and local.status == 0 and hasattr(engine, "trim"):  # keep the COO views only
        engine.trim([local.rows.data_ptr(), local.cols.data_ptr(), local.data.data_ptr()], build_ctx=True)
    line_base = np.concatenate([[0], np.cumsum([int(s[3]) for s in allst])])
    out = ShardResult(status=0, n_lines=int(line_base[-1]), n_records=int(sum(s[4] for s in allst)),
                      n_edges=int(sum(s[6] for s in allst)))
    parse_err = [k for k in range(world) if allst[k][0] != 0 and allst[k][0] not in CAST_ERRORS]
    cast_err = [k for k in range(world) if allst[k][0] in CAST_ERRORS]
    bad = parse_err[0] if parse_err else (cast_err[0] if cast_err else None)
    if first_unk is not None:
        gw = int(line_base[first_unk] + allst[first_unk][2])
        if bad is None or gw < int(line_base[bad] + allst[bad][1]) or allst[bad][0] in CAST_ERRORS:
            if not (bad == first_unk and allst[bad][0] == 8 and allst[bad][1] == allst[bad][2]):
                out.has_warning, out.warn_line = True, gw
                wb = torch.tensor([local.warn_byte if rank == first_unk else 0], dtype=torch.int64, device=dev)
                out.warn_byte = int(C.bcast(wb, first_unk).item())
    if bad is not None:
        out.status = int(allst[bad][0])
        if out.status in CAST_ERRORS:  # index in the global triplet stream
            trip_base = sum(int(allst[k][6]) * ktrip for k in range(bad))
            idx = torch.tensor([local.err_index if rank == bad else 0], dtype=torch.int64, device=dev)
            val = torch.tensor([local.err_value if rank == bad else 0.0], dtype=torch.float64, device=dev)
            out.err_index = trip_base + int(C.bcast(idx, bad).item())
            out.err_value = float(C.bcast(val, bad).item())
        else:
            out.err_line = int(line_base[bad] + allst[bad][1])
            out.n_records_before_error = int(sum(allst[k][4] for k in range(bad)) + allst[bad][5])
            det = torch.zeros(64, dtype=torch.uint8, device=dev)
            if rank == bad and local.err_detail:
                d = np.frombuffer(local.err_detail[:63], dtype=np.uint8)
                det[0] = len(d)
                det[1:1 + len(d)] = torch.from_numpy(d.copy()).to(dev)
            det = C.bcast(det, bad)
            k = int(det[0].item())
            out.err_detail = bytes(det[1:1 + k].cpu().numpy())
        return out
    out.n_records_before_error = out.n_records
    out.n_cast_overflow = int(sum(s[7] for s in allst))
    tm["local_build"] = (time.perf_counter() - t0) * 1e3
    for k, v in local.phase_ms.items():  # its device phases beside the host stages (diagnostics)
        tm["local_dev_" + k] = v

    if world == 1 and not force_protocol:  # one range: its local ids are the global ids
        out.n_nodes = local.n_local_nodes
        if gather_names:
            out.names_blob = local.names_blob.cpu().numpy()
            out.names_offsets = local.names_offsets.cpu().numpy()
        local.dtype_name = dtype
        if keep_coo:
            out.coo = (local.rows, local.cols, local.data)
        a, tstream = _route(engine, C, local, dtype, None, out.n_nodes, maxsym, not weight_tag, tm)
        return _finish(engine, C, out, a, tstream, maxsym, dtype, weight_tag, tm, int(local.rows.numel()), copy_out)

    # 3. names to owners, owner dedup in arrival (= global first-touch) order
    t1 = time.perf_counter()
    if world == 1:  # one owner: the keys stay where they are, in local-id order
        n_loc = int(local.n_local_nodes)
        pb, po = local.names_blob, local.names_offsets
        pidx = torch.arange(n_loc, dtype=torch.int32, device=dev)
        pst_l, po_l = [0, n_loc], [0, int(po[-1].item()) if n_loc else 0]
    else:
        pb, po, pidx, pst = engine.partition_keys(local.names_blob, local.names_offsets, world)
        if local.n_local_nodes:  # the owners' key and byte counts in one host read
            both = torch.cat([pst.to(torch.int64), po[pst.to(torch.int64)]]).tolist()
            pst_l, po_l = both[:world + 1], both[world + 1:]
        else:
            pst_l, po_l = pst.tolist(), [0] * (world + 1)
    tm["partition_keys"] = (time.perf_counter() - t1) * 1e3
    key_counts = [pst_l[k + 1] - pst_l[k] for k in range(world)]
    byte_counts = [int(po_l[k + 1] - po_l[k]) for k in range(world)]
    lens = (po[1:] - po[:-1]) if local.n_local_nodes else torch.zeros(0, dtype=torch.int64, device=dev)
    r_blob, _ = C.a2av(pb[:int(po_l[-1])] if local.n_local_nodes else pb[:0], byte_counts)
    # (the local ids travel as int32: order_keys widens the arrivals it reads)
    (r_lens, r_idx), r_kc = C.a2av_multi([lens, pidx], key_counts)
    r_off = torch.zeros(r_lens.numel() + 1, dtype=torch.int64, device=dev)
    if r_lens.numel():
        r_off[1:] = torch.cumsum(r_lens, 0)
    tm["key_exchange"] = (time.perf_counter() - t1) * 1e3 - tm["partition_keys"]
    t7 = time.perf_counter()
    if world == 1:  # one range: its local dictionary's keys are distinct already, in first-touch order
        nd = int(r_off.numel()) - 1
        ids = first_of = torch.arange(nd, dtype=torch.int32, device=dev)
    else:
        ids, first_of, nd = engine.dedup_keys(r_blob, r_off)
    tm["dedup_keys"] = (time.perf_counter() - t7) * 1e3
    # order key (source rank, local id) of each distinct key: global first-touch order
    dkey = (engine.order_keys(first_of, r_idx.to(torch.int64), r_kc) if nd and world > 1
            else r_idx[:0].to(torch.int64))
    tm["owner_dedup"] = (time.perf_counter() - t1) * 1e3

    # 4. global ids: rank of each distinct key's order key among all owners' (one owner: its order)
    t2 = time.perf_counter()
    if world > 1:
        all_dkey = C.allgather_v(dkey)
        n_global = int(sum(x.numel() for x in all_dkey))
        gid = engine.rank_keys(dkey, all_dkey, rank)
        del all_dkey
    else:
        n_global = nd
        gid = torch.arange(nd, dtype=torch.int64, device=dev)
    back, _ = C.a2av(gid[ids.to(torch.int64)].to(torch.int32) if nd else gid[:0].to(torch.int32), r_kc)
    gmap = None
    if rank > 0:  # rank 0's map is the identity (step 5)
        gmap = torch.empty(local.n_local_nodes, dtype=torch.int32, device=dev)
        if local.n_local_nodes:
            gmap[pidx.to(torch.int64)] = back
    tm["global_ids"] = (time.perf_counter() - t2) * 1e3
    if trim and hasattr(engine, "trim"):  # the dedup table and key partition: their outputs are tensors
        engine.trim()
    out.n_nodes = n_global
    if gather_names:
        # the owner's distinct keys (bytes at r_off[first_of]) with their global ids, to the
        # gathering rank(s) in one blob + lengths each; put in id order there (g2n_gather_names)
        t5 = time.perf_counter()
        d_lens = r_lens[first_of.to(torch.int64)] if nd else r_lens[:0]
        d_off = torch.zeros(nd + 1, dtype=torch.int64, device=dev)
        if nd:
            d_off[1:] = torch.cumsum(d_lens, 0)
        d_blob, _ = engine.gather_keys(r_blob, r_off, first_of, int(d_off[-1].item()))
        p_gid = list(C.parts(gid, root=names_root))
        p_len = list(C.parts(d_lens, root=names_root))
        p_blob = list(C.parts(d_blob, root=names_root))
        if p_gid:
            g_all = np.concatenate([x.cpu().numpy() for _, x in p_gid])
            l_all = np.concatenate([x.cpu().numpy() for _, x in p_len])
            b_all = np.concatenate([x.cpu().numpy() for _, x in p_blob])
            o_all = np.zeros(len(l_all) + 1, dtype=np.int64)
            np.cumsum(l_all, out=o_all[1:])
            # the key holding global id i; every id must be covered exactly once, or the protocol
            # is broken — raise here rather than hand g2n_gather_names an unchecked index
            if len(g_all) != n_global or (n_global and (g_all.min() < 0 or g_all.max() >= n_global)):
                raise RuntimeError(f"sharded names: {len(g_all)} ids gathered for {n_global} nodes")
            order = np.full(n_global, -1, dtype=np.int64)
            order[g_all] = np.arange(n_global, dtype=np.int64)
            if n_global and order.min() < 0:
                raise RuntimeError("sharded names: a global id was not gathered")
            out.names_blob, out.names_offsets = nat.gather_names(b_all, o_all, order)
        tm["names"] = (time.perf_counter() - t5) * 1e3

    # 5. the range's triplets over global ids (one gather per coordinate; the routes below need no
    #    map), to row owners (and the A.T stream for MAX-SYM); 6. this rank's CSR row slice
    t6 = time.perf_counter()
    local.dtype_name = dtype
    if rank > 0:  # rank 0's keys are the first n0 distinct keys in its own first-touch order: identity map
        local.rows, local.cols = engine.remap_pairs(local.rows, local.cols, gmap)
    tm["remap"] = (time.perf_counter() - t6) * 1e3
    if keep_coo:
        out.coo = (local.rows, local.cols, local.data)
    a, tstream = _route(engine, C, local, dtype, None, n_global, maxsym, not weight_tag, tm)
    return _finish(engine, C, out, a, tstream, maxsym, dtype, weight_tag, tm, int(local.rows.numel()), copy_out)


def _finish(engine, C, out, a, tstream, maxsym, dtype, weight_tag, tm, n_trip, copy_out=True):
    """Step 6 and the result's index-dtype count (scipy_index_dtype)."""
    row_lo, row_hi, indptr, indices, vals = _slice(engine, C, a, tstream, maxsym, out.n_nodes, dtype, weight_tag, tm,
                                                   copy_out)
    out.row_lo, out.row_hi = row_lo, row_hi
    out.indptr, out.indices, out.data = indptr, indices, vals
    nnz, trip = C.allreduce_sum([int(indices.numel()), n_trip], engine.device)
    out.index_maxval = nnz if maxsym else trip
    out.timings_ms = tm
    out.a2a_bytes_sent = C.sent
    return out


_NPDT = {"uint8": np.uint8, "int8": np.int8, "int32": np.int32, "float32": np.float32, "float64": np.float64}


def _np_dtype(t):
    return _NPDT[str(t.dtype).replace("torch.", "")]


def _bytes_view(t):
    """A tensor's raw bytes as a 1-D uint8 tensor (what the collectives move for any dtype)."""
    import torch

    t = t.contiguous().reshape(-1)
    return t if t.dtype == torch.uint8 else (t.view(torch.uint8) if t.numel() else t.to(torch.uint8))


def gather_coo(res: ShardResult, group=None, root=None):
    """Every rank's stream-order triplets concatenated in rank order (numpy): the file's
    stream-order COO (builders.py:281), since the ranges are contiguous.  On every rank (root
    None) or on `root` only (the others return None).  Index dtype from the shape (< 2^31 ids)."""
    C = Comm(group)
    rows, cols, data = res.coo
    npdt = _np_dtype(data)
    pr = [x.cpu().numpy() for _, x in C.parts(rows, root)]
    pc = [x.cpu().numpy() for _, x in C.parts(cols, root)]
    pd = [x.cpu().numpy().view(npdt) for _, x in C.parts(_bytes_view(data), root)]
    if not pr:
        return None
    return np.concatenate(pr), np.concatenate(pc), np.concatenate(pd)


def gather_csr(res: ShardResult, group=None, root=None):
    """The row slices concatenated into the full CSR (numpy) on every rank (root None: one
    broadcast per slice, no padding) or on `root` only (point-to-point; the others return None).
    indptr / indices take scipy's index dtype for the whole matrix (scipy_index_dtype: int64 once
    nnz — or the triplet count for coo.tocsr() — passes 2^31 - 1)."""
    C = Comm(group)
    idt = scipy_index_dtype(res.index_maxval, res.n_nodes)
    npdt = _np_dtype(res.data)
    parts_p = [x.cpu().numpy() for _, x in C.parts(res.indptr, root)]
    if not parts_p:
        for _ in C.parts(res.indices, root):
            pass
        for _ in C.parts(_bytes_view(res.data), root):
            pass
        return None
    indptr = concat_indptr(parts_p, idt)
    nnz = int(indptr[-1])
    indices = np.empty(nnz, dtype=idt)
    data = np.empty(nnz, dtype=npdt)
    pos = 0
    for _, x in C.parts(res.indices, root):
        k = x.numel()
        indices[pos:pos + k] = x.cpu().numpy()
        pos += k
    pos = 0
    for _, x in C.parts(_bytes_view(res.data), root):
        k = x.numel()
        data.view(np.uint8)[pos:pos + k] = x.cpu().numpy()
        pos += k
    return indptr, indices, data


# ------------------------------------------------------- sharded .gz: per-rank inflate --
def gz_member_at_or_after(path: str, off: int, size: int, window: int = 1 << 20) -> int:
    """The first gzip member start at or after byte `off` of a .gz file (RFC 1952: 1f 8b 08, reserved
    flag bits clear, and a header + first deflate bytes that zlib accepts), or `size` when there is
    none.  A false candidate inside compressed data is caught later: the slice before it does not
    inflate to a clean member chain (gz_rank_text)."""
    import zlib

    if off <= 0:
        return 0
    with open(path, "rb") as fh:
        fd = fh.fileno()
        pos = off
        while pos < size:
            blk = os.pread(fd, window + 2, pos)
            k = 0
            while True:
                k = blk.find(b"\x1f\x8b\x08", k)
                if k < 0 or k >= window:
                    break
                cand = pos + k
                head = os.pread(fd, 1 << 16, cand)
                if len(head) >= 10 and head[3] & 0xE0 == 0:
                    try:
                        zlib.decompressobj(31).decompress(head, 1 << 16)
                        return cand
                    except zlib.error:
                        pass
                k += 1
            pos += window
    return size


def gz_rank_text(path: str, engine, group=None):
    """This rank's line-aligned range of a multi-member / BGZF .gz, inflating only the members that
    start in its share of the compressed bytes (every rank inflated the whole file).

    1. rank r takes the members starting in [r * size / G, (r + 1) * size / G) of the compressed file
       (gz_member_at_or_after at both ends: every rank finds the same cut points) and inflates that
       slice on its host (g2n_gunzip: member-parallel) — each slice a clean member chain, so together
       they are the whole file's chain (gzip.py's reader sees the same bytes);
    2. the ranks' text lengths are all-gathered: the inflated stream's line-aligned split points
       (shard.line_ranges' rule — the first line start at or after r * N / G) are found from what each
       rank reports about its own text (the byte before a split, the first newline at or after it);
    3. one all-to-all-v moves the bytes to their owners (on the GPU with RCCL): rank r ends with
       exactly the range line_ranges would give it over the whole inflated file.
    Returns (device uint8 tensor, inflated bytes) — or None on every rank when any slice does not
    inflate cleanly (a false member candidate, corruption, a single huge member cut by a candidate):
    the caller then takes the whole-file path, whose exact reader raises gzip.py's errors."""
    import torch

    C = Comm(group)
    world, rank = C.world, C.rank
    size = os.path.getsize(path)
    c0 = gz_member_at_or_after(path, rank * size // world, size)
    c1 = gz_member_at_or_after(path, (rank + 1) * size // world, size) if rank + 1 < world else size
    text, ok = b"", 1
    if c1 > c0:
        with open(path, "rb") as fh:
            blob = os.pread(fh.fileno(), c1 - c0, c0)
        try:
            text, _ = nat.gunzip(blob)
        except (nat.GzipFailure, RuntimeError):
            ok = 0
        del blob
    lens = C.allgather_list([len(text), ok])
    if not all(x[1] for x in lens):
        return None
    n_r = [int(x[0]) for x in lens]
    P = np.concatenate([[0], np.cumsum(n_r)]).astype(np.int64)
    N = int(P[-1])
    arr = np.frombuffer(text, dtype=np.uint8)
    # 2. what this rank knows about each nominal split m_k = k N / G: the byte before it, and the
    #    first newline at or after it inside this rank's text (-1: none here)
    rep = []
    for k in range(1, world):
        m = k * N // world
        before = int(arr[m - 1 - P[rank]]) if P[rank] <= m - 1 < P[rank + 1] else -1
        nl = -1
        lo = max(m, int(P[rank])) - int(P[rank])
        if lo < len(arr):
            pos, win = lo, 1 << 16
            while pos < len(arr):
                hit = np.flatnonzero(arr[pos:pos + win] == 0x0A)
                if len(hit):
                    nl = int(P[rank]) + pos + int(hit[0])
                    break
                pos += win
                win = min(win * 2, 1 << 26)
        rep += [before, nl]
    allrep = C.allgather_list(rep) if world > 1 else [rep]
    starts = [0]
    for k in range(1, world):
        m = k * N // world
        before = max(r[2 * (k - 1)] for r in allrep)
        nls = [r[2 * (k - 1) + 1] for r in allrep if r[2 * (k - 1) + 1] >= 0]
        if m <= 0 or m >= N or before == 0x0A:
            s = min(max(m, 0), N)
        else:
            s = min(nls) + 1 if nls else N
        starts.append(max(s, starts[-1]))
    starts.append(N)
    # 3. the bytes of [P_r, P_r + n_r) to the ranks whose [starts_k, starts_k+1) they overlap
    send = [max(0, min(int(P[rank + 1]), starts[k + 1]) - max(int(P[rank]), starts[k])) for k in range(world)]
    t = torch.from_numpy(arr.copy()) if len(arr) else torch.zeros(0, dtype=torch.uint8)
    t = t.to(engine.device)
    del text, arr
    got, _ = C.a2av(t, send)
    return got.to(engine.device), N
