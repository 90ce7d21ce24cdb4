"""ctypes binding of libg2n.so (include/g2n.h) — the only way Python reaches the GPU path.

The library is built in-tree (gfa2network_amd/_lib/libg2n.so, ``make -C
gfa2network_amd/csrc`` or ``__graft_entry__.build()``).  There is no fallback: if the
library or a HIP device is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import sys
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

LIB_PATH = Path(__file__).resolve().parent / "_lib" / "libg2n.so"

ABI_VERSION = 2
MAX_PHASES = 40

# status codes (include/g2n.h)
OK = 0
E_MALFORMED_L, E_MALFORMED_E, E_MALFORMED_C, E_MALFORMED_P, E_MALFORMED_O = 1, 2, 3, 4, 5
E_INDEX_LIST, E_INDEX_BYTES, E_UNICODE, E_INT_TOO_LARGE = 6, 7, 8, 9
E_CAST_OVERFLOW, E_CAST_INF, E_CAST_NAN = 10, 11, 12
E_ARG, E_IO, E_GZIP, E_DEVICE, E_NOMEM, E_UNSUPPORTED = 13, 14, 15, 16, 17, 18

DTYPE_CODES = {"bool": 0, "int8": 1, "int32": 2, "float32": 3, "float64": 4}
CODE_DTYPES = {v: np.dtype(k) for k, v in DTYPE_CODES.items()}
OUT_PARSE, OUT_CSR, OUT_COO, OUT_EDGE_LIST = 0, 1, 2, 3
FMT_COO, FMT_CSR, FMT_TEXT = 0, 1, 2

# every symbol include/g2n.h declares (tests check the library exports all of them)
EXPORTED = [
    "g2n_version", "g2n_abi_version", "g2n_options_init", "g2n_device_count", "g2n_device_memory", "g2n_last_error",
    "g2n_status_name", "g2n_release_shared", "g2n_build_from_path", "g2n_build_from_buffer", "g2n_result_free",
    "g2n_coo_to_csr", "g2n_coo_to_csr_band", "g2n_context_create", "g2n_context_destroy", "g2n_context_stream", "g2n_context_trim",
    "g2n_build_device", "g2n_build_decimal_range", "g2n_count_device", "g2n_order_keys", "g2n_rank_keys", "g2n_upload_file_range", "g2n_partition_keys", "g2n_dedup_keys", "g2n_gather_keys", "g2n_remap_pairs", "g2n_route_triplets", "g2n_csr_from_coo_pair",
    "g2n_context_group_slots", "g2n_route_group_slots", "g2n_csr_from_group_slots",
    "g2n_keyset_create", "g2n_keyset_add", "g2n_keyset_view", "g2n_keyset_free",
    "g2n_gunzip", "g2n_gunzip_chunked", "g2n_free", "g2n_split_render", "g2n_split_get", "g2n_split_segments", "g2n_split_free", "g2n_join_names", "g2n_gather_names", "g2n_write_npz", "g2n_write_node_map", "g2n_first_bad_utf8",
]


# options.test_flags (include/g2n.h G2N_TEST_*): the builds of this process take normally-rare
# paths when a test sets them; 0 in every real use
TEST_NO_BUCKETS = 2      # MAX-SYM through the general row-sum path
TEST_NO_LEAN = 4         # decimal ids without the lean parse (ids per touch, then k_triplets)
TEST_DICT_HASH = 8       # no decimal ids, no direct-address tier: the hash dictionary tiers
TEST_DICT_GENERAL = 16   # no decimal ids, no S-first fast path: the general insert rounds
TEST_NO_TILE_LOCAL = 32  # decimal ids: the lean parse after K1's tile bases, not the tile-local pass
TEST_HOST_INFLATE = 64   # a BGZF ".gz" read by the host gzip readers instead of the GPU inflate
TEST_NO_GROUP = 128      # tile-local parse into per-tile slots + compaction (never group slots)
TEST_NO_HASH_LEAN = 256  # names that are not decimal ids: the classic hash tiers, never the lean S-first one
TEST_THROW_AFTER_IDS = 512  # the build throws (G2N_E_DEVICE) once its ids and names are set up: call-state tests
TEST_INDEX64 = 1024      # unweighted CSR results in int64 indptr / indices (the > 2^31 - 1 entries path)
TEST_DICT_DIRECT = 2048  # decimal ids in S order through the direct-address tier (not the decimal-id parse)
TEST_NO_DIRECT = 4096    # never the direct-address tier: the lean hash tier instead
TEST_NO_EXT_LEAN = 8192  # bidirected / weighted decimal builds through K1 + the lean parse (not tile-local)
TEST_NO_DEC_TEXT = 16384  # edge-list export of decimal ids through the names blob (not the arithmetic render)
TEST_NO_DEC_PREFIX = 32768  # prefixed names "P1".."PN" in S order through the direct tier (not the tile-local parse)
TEST_FLAGS = int(os.environ.get("G2N_TEST_FLAGS", "0"), 0)  # (diagnostics: force the paths below for a whole run)
# options.range_flags (include/g2n.h G2N_RANGE_*): set by the sharded / chunked protocol (shard.py)
RANGE_DECIMAL = 1        # this byte range's ids are global decimals (range_s_base / range_n_segments)
RANGE_EVIDENCE = 2       # report the range's evidence instead of checking (g2n_build_decimal_range sets it)
RANGE_NO_VALUES = 4      # coordinates only: values left unwritten
RANGE_SLOTS = 8          # with DECIMAL + NO_VALUES: the COO stays in the parse's group slots (no compaction)


class Options(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_uint32),
        ("directed", ctypes.c_int32),
        ("bidirected", ctypes.c_int32),
        ("keep_directed_bidir", ctypes.c_int32),
        ("asymmetric", ctypes.c_int32),
        ("strip_orientation", ctypes.c_int32),
        ("dtype", ctypes.c_int32),
        ("output", ctypes.c_int32),
        ("weight_tag", ctypes.c_char_p),
        ("want_node_names", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("unknown_warned", ctypes.c_int32),
        ("range_flags", ctypes.c_int32),
        ("range_s_base", ctypes.c_int64),
        ("range_n_segments", ctypes.c_int64),
        ("test_flags", ctypes.c_uint32),
        ("reserved_", ctypes.c_int32 * 3),
    ]


class Result(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_uint32),
        ("status", ctypes.c_int32),
        ("err_line", ctypes.c_int64),
        ("err_index", ctypes.c_int64),
        ("err_value", ctypes.c_double),
        ("err_detail", ctypes.c_void_p),
        ("err_detail_len", ctypes.c_int64),
        ("has_warning", ctypes.c_int32),
        ("warn_byte", ctypes.c_int32),
        ("warn_line", ctypes.c_int64),
        ("n_lines", ctypes.c_int64),
        ("n_records", ctypes.c_int64),
        ("n_records_before_error", ctypes.c_int64),
        ("n_edges", ctypes.c_int64),
        ("n_nodes", ctypes.c_int64),
        ("names_blob", ctypes.c_void_p),
        ("names_offsets", ctypes.c_void_p),
        ("format", ctypes.c_int32),
        ("dtype", ctypes.c_int32),
        ("index_width", ctypes.c_int32),
        ("sum_sorted", ctypes.c_int32),
        ("nnz", ctypes.c_int64),
        ("rows", ctypes.c_void_p),
        ("cols", ctypes.c_void_p),
        ("indptr", ctypes.c_void_p),
        ("indices", ctypes.c_void_p),
        ("data", ctypes.c_void_p),
        ("names_bytes", ctypes.c_uint64),
        ("n_cast_overflow", ctypes.c_int64),
        ("input_bytes", ctypes.c_uint64),
        ("n_phases", ctypes.c_int32),
        ("sum_t_sorted", ctypes.c_int32),
        ("phase_ms", ctypes.c_double * MAX_PHASES),
        ("phase_names", ctypes.c_char_p * MAX_PHASES),
        ("host_ms_read", ctypes.c_double),
        ("host_ms_h2d", ctypes.c_double),
        ("host_ms_d2h", ctypes.c_double),
        ("priv_", ctypes.c_void_p),
    ]


_lib = None


class NativeUnavailable(RuntimeError):
    """libg2n.so is missing or cannot be loaded (the path has no CPU fallback)."""


def _torch_hip_runtime() -> str | None:
    """Path of the HIP runtime bundled in the installed torch wheel, found without importing torch."""
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError, AttributeError):
        return None
    if spec is None or not spec.origin:
        return None
    p = Path(spec.origin).parent / "lib" / "libamdhip64.so"
    return str(p) if p.exists() else None


def _preload_hip_runtime() -> None:
    """One HIP runtime per process: torch's wheel bundles a libamdhip64.so.7 of its own (same
    SONAME as /opt/rocm's, which libg2n.so names), and whichever loads first serves both; torch
    cannot initialise the device on /opt/rocm's.  So when torch is installed, its runtime is
    loaded by path (RTLD_GLOBAL) before libg2n.so — without importing torch, which the
    single-GPU path never needs; with no torch, libg2n.so resolves /opt/rocm's."""
    if "torch" in sys.modules and sys.modules["torch"] is not None:
        return  # torch loaded its runtime already
    p = _torch_hip_runtime()
    if p:
        try:
            ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        except OSError:
            pass


def hip_runtime() -> ctypes.CDLL:
    """The HIP runtime libg2n.so runs on (by its SONAME: whichever libamdhip64.so.7 the process
    loaded — torch's when torch is installed), for callers that copy device memory themselves."""
    load()
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipMemcpy.restype = ctypes.c_int
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipMalloc.restype = ctypes.c_int
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipFree.restype = ctypes.c_int
    hip.hipSetDevice.argtypes = [ctypes.c_int]
    hip.hipSetDevice.restype = ctypes.c_int
    return hip


def load() -> ctypes.CDLL:
    """Load libg2n.so once; raise NativeUnavailable when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("G2N_LIB", str(LIB_PATH))
    if not Path(path).exists():
        raise NativeUnavailable(
            f"{path} not found: build it with `make -C gfa2network_amd/csrc` "
            "(or __graft_entry__.build()); the GFA->CSR path has no CPU fallback")
    _preload_hip_runtime()
    try:
        lib = ctypes.CDLL(path)
    except OSError as exc:  # pragma: no cover - depends on the image
        raise NativeUnavailable(f"cannot load {path}: {exc}") from exc
    lib.g2n_version.restype = ctypes.c_char_p
    lib.g2n_abi_version.restype = ctypes.c_uint32
    lib.g2n_last_error.restype = ctypes.c_char_p
    lib.g2n_status_name.restype = ctypes.c_char_p
    lib.g2n_status_name.argtypes = [ctypes.c_int]
    lib.g2n_options_init.argtypes = [ctypes.POINTER(Options)]
    lib.g2n_options_init.restype = None
    lib.g2n_device_count.restype = ctypes.c_int
    lib.g2n_device_memory.argtypes = [ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    lib.g2n_device_memory.restype = ctypes.c_int
    lib.g2n_build_from_path.argtypes = [ctypes.c_char_p, ctypes.POINTER(Options),
                                        ctypes.POINTER(ctypes.POINTER(Result))]
    lib.g2n_build_from_path.restype = ctypes.c_int
    lib.g2n_build_from_buffer.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(Options),
                                          ctypes.POINTER(ctypes.POINTER(Result))]
    lib.g2n_build_from_buffer.restype = ctypes.c_int
    lib.g2n_result_free.argtypes = [ctypes.POINTER(Result)]
    lib.g2n_result_free.restype = None
    lib.g2n_coo_to_csr.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                   ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.c_int32, ctypes.c_uint32, ctypes.POINTER(ctypes.POINTER(Result))]
    lib.g2n_coo_to_csr.restype = ctypes.c_int
    lib.g2n_coo_to_csr_band.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                        ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_int32, ctypes.POINTER(ctypes.POINTER(Result))]
    lib.g2n_coo_to_csr_band.restype = ctypes.c_int
    lib.g2n_context_create.argtypes = [ctypes.c_int]
    lib.g2n_context_create.restype = ctypes.c_void_p
    lib.g2n_context_destroy.argtypes = [ctypes.c_void_p]
    lib.g2n_context_destroy.restype = None
    lib.g2n_context_stream.argtypes = [ctypes.c_void_p]
    lib.g2n_context_stream.restype = ctypes.c_void_p
    lib.g2n_context_trim.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint64,
                                     ctypes.POINTER(ctypes.c_uint64)]
    lib.g2n_context_trim.restype = ctypes.c_int
    lib.g2n_build_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.POINTER(Options), ctypes.POINTER(Result)]
    lib.g2n_build_device.restype = ctypes.c_int
    P, U64, I32, U32, I64 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32, ctypes.c_uint32, ctypes.c_int64
    lib.g2n_partition_keys.argtypes = [P, P, U64, P, U64, U32, P, P, P, P]
    lib.g2n_dedup_keys.argtypes = [P, P, U64, P, U64, P, P, ctypes.POINTER(U64)]
    lib.g2n_gather_keys.argtypes = [P, P, P, P, U64, P, U64, P, ctypes.POINTER(U64)]
    lib.g2n_remap_pairs.argtypes = [P, P, U64, P, P, U64]
    lib.g2n_route_triplets.argtypes = [P, P, P, P, U64, I32, P, U64, U32, I32, P, P, P, P]
    lib.g2n_csr_from_coo_pair.argtypes = [P, P, P, P, U64, P, P, P, U64, I32, I64, U64, U64, I32, I32, I32,
                                          ctypes.POINTER(Result)]
    lib.g2n_release_shared.argtypes = [I32, ctypes.POINTER(U64)]
    lib.g2n_release_shared.restype = ctypes.c_int
    lib.g2n_context_group_slots.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(U64), ctypes.POINTER(U64)]
    lib.g2n_route_group_slots.argtypes = [P, P, P, P, U64, U64, U64, U64, U32, I32, P, P, P]
    lib.g2n_csr_from_group_slots.argtypes = [P, P, P, P, U64, U64, U64, I32, U64, I32, ctypes.POINTER(Result)]
    lib.g2n_gunzip.argtypes = [P, ctypes.c_size_t, I32, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t),
                               ctypes.POINTER(I32), ctypes.POINTER(I32)]
    lib.g2n_gunzip.restype = ctypes.c_int
    lib.g2n_gunzip_chunked.argtypes = [P, ctypes.c_size_t, ctypes.c_size_t, ctypes.POINTER(P),
                                       ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(I32)]
    lib.g2n_gunzip_chunked.restype = ctypes.c_int
    lib.g2n_free.argtypes = [P]
    lib.g2n_split_render.argtypes = [P, ctypes.c_size_t, I32, ctypes.POINTER(P)]
    lib.g2n_split_render.restype = ctypes.c_int
    PP, PU = ctypes.POINTER(P), ctypes.POINTER(U64)
    lib.g2n_split_get.argtypes = [P, PP, PU, PP, PP, PU, PP, PP, PP, PU, ctypes.POINTER(I32)]
    lib.g2n_split_get.restype = None
    lib.g2n_split_segments.argtypes = [P, PP, PU]
    lib.g2n_split_segments.restype = None
    lib.g2n_split_free.argtypes = [P]
    lib.g2n_join_names.argtypes = [P, P, U64, ctypes.c_uint8, P]
    lib.g2n_join_names.restype = ctypes.c_int
    lib.g2n_gather_names.argtypes = [P, P, P, U64, P, P]
    lib.g2n_gather_names.restype = ctypes.c_int
    lib.g2n_write_npz.argtypes = [ctypes.c_char_p, I32, P, P, P, P, P, I32]
    lib.g2n_write_npz.restype = ctypes.c_int
    lib.g2n_write_node_map.argtypes = [ctypes.c_char_p, P, P, U64, I32, ctypes.POINTER(I64)]
    lib.g2n_write_node_map.restype = ctypes.c_int
    lib.g2n_first_bad_utf8.argtypes = [P, P, U64]
    lib.g2n_first_bad_utf8.restype = I64
    lib.g2n_upload_file_range.argtypes = [ctypes.c_char_p, U64, U64, P, I32]
    lib.g2n_count_device.argtypes = [P, P, ctypes.c_size_t, ctypes.POINTER(I64)]
    lib.g2n_build_decimal_range.argtypes = [P, P, ctypes.c_size_t, ctypes.POINTER(Options), ctypes.POINTER(I64),
                                            ctypes.POINTER(Result)]
    lib.g2n_order_keys.argtypes = [P, P, P, U64, P, U32, P]
    lib.g2n_rank_keys.argtypes = [P, P, U64, P, P, U32, U32, P]
    lib.g2n_keyset_create.argtypes = [P, ctypes.POINTER(P)]
    lib.g2n_keyset_add.argtypes = [P, P, U64, P, U64, P, ctypes.POINTER(U64)]
    lib.g2n_keyset_view.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(U64), ctypes.POINTER(U64)]
    lib.g2n_keyset_free.argtypes = [P]
    lib.g2n_keyset_free.restype = None
    for f in ("g2n_keyset_create", "g2n_keyset_add", "g2n_keyset_view", "g2n_partition_keys", "g2n_dedup_keys", "g2n_gather_keys", "g2n_remap_pairs", "g2n_route_triplets", "g2n_csr_from_coo_pair",
              "g2n_context_group_slots", "g2n_route_group_slots", "g2n_csr_from_group_slots",
              "g2n_upload_file_range", "g2n_count_device", "g2n_build_decimal_range", "g2n_order_keys",
              "g2n_rank_keys"):
        getattr(lib, f).restype = ctypes.c_int
    if lib.g2n_abi_version() != ABI_VERSION:
        raise NativeUnavailable("libg2n.so ABI version mismatch; rebuild it")
    _lib = lib
    return lib


def last_error() -> str:
    return load().g2n_last_error().decode(errors="replace")


def status_name(code: int) -> str:
    return load().g2n_status_name(code).decode()


def make_options(*, directed=True, bidirected=False, keep_directed_bidir=False, asymmetric=False,
                 strip_orientation=False, dtype="float64", weight_tag=None, output=OUT_PARSE,
                 want_node_names=True, device=0, test_flags=None) -> Options:
    lib = load()
    o = Options()
    lib.g2n_options_init(ctypes.byref(o))
    o.directed = int(bool(directed))
    o.bidirected = int(bool(bidirected))
    o.keep_directed_bidir = int(bool(keep_directed_bidir))
    o.asymmetric = int(bool(asymmetric))
    o.strip_orientation = int(bool(strip_orientation))
    o.dtype = DTYPE_CODES[dtype]
    o.output = output
    o.weight_tag = weight_tag.encode("utf-8") if weight_tag else None
    o.want_node_names = int(bool(want_node_names))
    o.device = int(device)
    # tests only: force a normally rare path (same results); include/g2n.h G2N_TEST_*
    o.test_flags = int(TEST_FLAGS if test_flags is None else test_flags)
    return o


class _Owner:
    """Frees one g2n_result when the last numpy view of its buffers goes away."""

    def __init__(self, ptr):
        self.ptr = ptr

    def __del__(self):
        if self.ptr is not None and _lib is not None:
            _lib.g2n_result_free(self.ptr)
            self.ptr = None


def _view(addr: int | None, count: int, dtype, owner: _Owner) -> np.ndarray:
    """Zero-copy numpy view of library-owned host memory, keeping `owner` alive."""
    dtype = np.dtype(dtype)
    if not addr or count == 0:
        return np.zeros(0, dtype=dtype)
    buf = (ctypes.c_uint8 * (count * dtype.itemsize)).from_address(addr)
    buf._g2n_owner = owner  # the ctypes buffer (the array's base) pins the result
    return np.frombuffer(buf, dtype=dtype, count=count)


@dataclass
class RawResult:
    """What one native build returned, before it is turned into scipy objects."""

    status: int = 0
    message: str = ""
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
    names_blob: np.ndarray | None = None
    names_offsets: np.ndarray | None = None
    format: str = "coo"
    dtype: np.dtype = field(default_factory=lambda: np.dtype("float64"))
    rows: np.ndarray | None = None
    cols: np.ndarray | None = None
    indptr: np.ndarray | None = None
    indices: np.ndarray | None = None
    data: np.ndarray | None = None
    sum_sorted: bool = True
    sum_buckets: bool = False  # the CSR came from the bucket partition (g2n_sym.hip), not the row sums
    n_cast_overflow: int = 0
    input_bytes: int = 0
    phase_ms: dict = field(default_factory=dict)
    host_ms: dict = field(default_factory=dict)


def _from_result(ptr, rc: int) -> RawResult:
    if not ptr:
        raise RuntimeError(f"{status_name(rc)}: {last_error()}")
    r = ptr.contents
    owner = _Owner(ptr)
    out = RawResult(status=r.status, message=last_error() if r.status else "")
    out.err_line, out.err_index, out.err_value = r.err_line, r.err_index, r.err_value
    if r.err_detail and r.err_detail_len:
        out.err_detail = ctypes.string_at(r.err_detail, r.err_detail_len)
    out.has_warning, out.warn_byte, out.warn_line = bool(r.has_warning), r.warn_byte, r.warn_line
    out.n_lines, out.n_records = r.n_lines, r.n_records
    out.n_records_before_error, out.n_edges, out.n_nodes = r.n_records_before_error, r.n_edges, r.n_nodes
    out.dtype = CODE_DTYPES.get(r.dtype, np.dtype("float64"))
    out.sum_sorted = bool(r.sum_sorted)
    out.sum_buckets = r.sum_sorted < 0
    out.n_cast_overflow = int(r.n_cast_overflow)
    out.input_bytes = int(r.input_bytes)
    if r.format == FMT_TEXT and r.data:
        out.format = "text"  # export --format edge-list: the rendered lines (all, or those before a failure)
        out.data = _view(r.data, r.nnz, np.uint8, owner)
    elif r.status == OK:
        idx = np.int32 if r.index_width == 4 else np.int64
        if r.names_offsets:
            out.names_offsets = _view(r.names_offsets, r.n_nodes + 1, np.int64, owner)
            out.names_blob = _view(r.names_blob, int(out.names_offsets[-1]), np.uint8, owner)
        if r.format == FMT_COO:
            out.format = "coo"
            out.rows = _view(r.rows, r.nnz, idx, owner)
            out.cols = _view(r.cols, r.nnz, idx, owner)
        else:
            out.format = "csr"
            out.indptr = _view(r.indptr, r.n_nodes + 1, idx, owner)
            out.indices = _view(r.indices, r.nnz, idx, owner)
        out.data = _view(r.data, r.nnz, out.dtype, owner)
    for k in range(r.n_phases):  # repeated phases (e.g. several insert rounds) add up
        name = r.phase_names[k].decode()
        if not name.startswith("_"):
            out.phase_ms[name] = out.phase_ms.get(name, 0.0) + r.phase_ms[k]
    out.host_ms = {"read": r.host_ms_read, "h2d": r.host_ms_h2d, "d2h": r.host_ms_d2h}
    return out


def build_from_path(path: str, opts: Options) -> RawResult:
    lib = load()
    res = ctypes.POINTER(Result)()
    rc = lib.g2n_build_from_path(os.fsencode(path), ctypes.byref(opts), ctypes.byref(res))
    return _from_result(res, rc)


def build_from_buffer(data: bytes | bytearray | memoryview | np.ndarray, opts: Options) -> RawResult:
    lib = load()
    arr = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    res = ctypes.POINTER(Result)()
    rc = lib.g2n_build_from_buffer(arr.ctypes.data if arr.size else None, arr.size, ctypes.byref(opts),
                                   ctypes.byref(res))
    return _from_result(res, rc)


BAND_ENTRIES = 2**31 - 2  # entries one g2n_coo_to_csr_band call takes (the weighted row-sum path's limit)


def coo_to_csr(rows: np.ndarray, cols: np.ndarray, data: np.ndarray, n_rows: int, n_cols: int,
               device: int = 0, test_flags: int | None = None, band_entries: int | None = None) -> RawResult:
    """scipy coo.tocsr() on the GPU (g2n_coo_to_csr): indptr / indices in scipy's index dtype
    (int64 past 2^31 - 1 entries).  A COO past what one call takes (a weighted matrix past 2^31 - 2
    entries, any past 2^32 - 2) is converted in row bands (_coo_to_csr_bands); band_entries forces
    bands of at most that many entries (tests)."""
    lib = load()
    dt = np.dtype(data.dtype)
    if dt.name not in DTYPE_CODES:
        raise NotImplementedError(f"GPU COO->CSR supports {sorted(DTYPE_CODES)}, not {dt}")
    if max(n_rows, n_cols) >= 2**31 - 1:
        raise NotImplementedError("GPU COO->CSR needs node ids below 2^31 - 1")
    r = np.ascontiguousarray(rows, dtype=np.int32)
    c = np.ascontiguousarray(cols, dtype=np.int32)
    d = np.ascontiguousarray(data)
    flags = TEST_FLAGS if test_flags is None else test_flags
    if band_entries is not None:
        return _coo_to_csr_bands(r, c, d, n_rows, n_cols, device, band_entries)
    if flags & TEST_INDEX64 and len(d) and not bool(np.all(d == 1)):
        # the past-2^31 route of a weighted COO on a small input: three row bands, int64 indices
        return _coo_to_csr_bands(r, c, d, n_rows, n_cols, device, len(d) // 3 + 1, index64=True)
    res = ctypes.POINTER(Result)()
    rc = lib.g2n_coo_to_csr(r.ctypes.data, c.ctypes.data, d.ctypes.data, len(d), n_rows, n_cols, 4,
                            DTYPE_CODES[dt.name], device, flags, ctypes.byref(res))
    if rc == E_NOMEM and release_shared(device):  # once more without what caches held
        rc = lib.g2n_coo_to_csr(r.ctypes.data, c.ctypes.data, d.ctypes.data, len(d), n_rows, n_cols, 4,
                                DTYPE_CODES[dt.name], device, flags, ctypes.byref(res))
    if rc == E_UNSUPPORTED and len(d) > BAND_ENTRIES:  # past one call's limit: row bands
        return _coo_to_csr_bands(r, c, d, n_rows, n_cols, device, BAND_ENTRIES)
    if rc == E_UNSUPPORTED:  # a documented size limit (include/g2n.h)
        raise NotImplementedError(f"GPU COO->CSR: {last_error()}")
    out = _from_result(res, rc)
    if out.status != OK:
        raise RuntimeError(f"{status_name(out.status)}: {out.message}")
    return out


def _coo_to_csr_bands(r, c, d, n_rows: int, n_cols: int, device: int, limit: int, index64: bool = False) -> RawResult:
    """coo.tocsr() (utils.py:55) of a COO too large for one g2n_coo_to_csr call, in row bands of at most
    `limit` entries (g2n_coo_to_csr_band).  Each band's triplets keep their stream order (a stable
    selection), so each row's duplicates meet in scipy's order; scipy's has_sorted_indices verdict is
    the whole matrix's — when some band holds an unsorted row, csr_sort_indices reorders every row —
    so bands that were sorted on their own are re-run with the matrix's verdict.  indptr / indices in
    scipy's dtype for the whole COO (int64 once its entries pass 2^31 - 1: _coo_to_compressed)."""
    lib = load()
    n = len(d)
    dt = np.dtype(d.dtype)
    counts = np.bincount(r, minlength=n_rows) if n else np.zeros(n_rows, dtype=np.int64)
    if n_rows and int(counts.max()) > limit:
        raise NotImplementedError("GPU COO->CSR: a row holds more entries than one band takes")
    cum = np.cumsum(counts, dtype=np.int64)
    cuts = [0]
    while cuts[-1] < n_rows:
        base = int(cum[cuts[-1] - 1]) if cuts[-1] else 0
        nxt = int(np.searchsorted(cum, base + limit, side="right"))
        cuts.append(min(max(nxt, cuts[-1] + 1), n_rows))
    if n_rows == 0:
        cuts.append(0)
    bands = list(zip(cuts[:-1], cuts[1:]))

    def run(lo, hi, force):
        sel = np.flatnonzero((r >= lo) & (r < hi)) if len(bands) > 1 else None
        br = (r[sel] - lo) if sel is not None else r
        bc, bd = (c[sel], d[sel]) if sel is not None else (c, d)
        br = np.ascontiguousarray(br, dtype=np.int32)
        bc, bd = np.ascontiguousarray(bc), np.ascontiguousarray(bd)
        res = ctypes.POINTER(Result)()
        rc = lib.g2n_coo_to_csr_band(br.ctypes.data, bc.ctypes.data, bd.ctypes.data, len(bd), hi - lo, n_cols,
                                     DTYPE_CODES[dt.name], device, force, ctypes.byref(res))
        if rc == E_NOMEM and release_shared(device):  # once more without what caches held
            rc = lib.g2n_coo_to_csr_band(br.ctypes.data, bc.ctypes.data, bd.ctypes.data, len(bd), hi - lo, n_cols,
                                         DTYPE_CODES[dt.name], device, force, ctypes.byref(res))
        if rc == E_UNSUPPORTED:
            raise NotImplementedError(f"GPU COO->CSR band: {last_error()}")
        out = _from_result(res, rc)
        if out.status != OK:
            raise RuntimeError(f"{status_name(out.status)}: {out.message}")
        # (copies: the next band's call reuses the context the result views point into)
        return (np.array(out.indptr), np.array(out.indices), np.array(out.data),
                None if out.sum_buckets else not out.sum_sorted)

    parts = [run(lo, hi, -1) for lo, hi in bands]
    if any(p[3] is True for p in parts):  # the matrix is unsorted: scipy sorts every row of it
        parts = [run(lo, hi, 1) if p[3] is False else p for (lo, hi), p in zip(bands, parts)]
    idt = np.int64 if index64 or max(n, n_rows) > 2**31 - 1 else np.int32
    nnz = sum(len(p[1]) for p in parts)
    indptr = np.empty(n_rows + 1, dtype=idt)
    indices = np.empty(nnz, dtype=idt)
    vals = np.empty(nnz, dtype=dt)
    indptr[0] = 0
    pos = 0
    for (lo, hi), p in zip(bands, parts):
        k = len(p[1])
        indptr[lo + 1:hi + 1] = p[0][1:].astype(np.int64) + pos
        indices[pos:pos + k] = p[1]
        vals[pos:pos + k] = p[2]
        pos += k
    out = RawResult(status=OK, format="csr", dtype=dt, n_nodes=n_rows, indptr=indptr, indices=indices, data=vals)
    out.sum_sorted = not any(p[3] is True for p in parts)
    return out


def host_bytes_at(addr: int, n: int) -> bytes:
    """bytes copy of n bytes at addr (ctypes.string_at truncates its size to a C int)."""
    if not n:
        return b""
    return (ctypes.c_char * n).from_address(addr).raw


def gunzip_chunked(data: bytes, chunk_bytes: int = 0) -> tuple[bytes, int] | None:
    """The chunk-parallel single-member inflate alone: (bytes, chunks that decoded from a block
    start of their own), or None when it declines."""
    lib = load()
    arr = np.frombuffer(data, dtype=np.uint8)
    if not arr.size:
        return None
    out, n, chunks = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_int32()
    rc = lib.g2n_gunzip_chunked(arr.ctypes.data, arr.size, chunk_bytes, ctypes.byref(out), ctypes.byref(n),
                                ctypes.byref(chunks))
    if rc == E_UNSUPPORTED:
        return None
    if rc != OK:
        raise RuntimeError(f"{status_name(rc)}: {last_error()}")
    try:
        return host_bytes_at(out.value, n.value), int(chunks.value)
    finally:
        lib.g2n_free(out)


def split_render(data, bidirected: bool):
    """g2n_split_render: (text, names_blob, names_offsets, warnings [(kind, segment bytes)],
    many_nodes, intervals per segment) for parse_gfa(..., split_on_alignment=True)
    (api._parse_gfa_split)."""
    lib = load()
    arr = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data,
                               dtype=np.uint8)
    h = ctypes.c_void_p()
    rc = lib.g2n_split_render(arr.ctypes.data if arr.size else None, arr.size, int(bool(bidirected)), ctypes.byref(h))
    if rc != OK:
        raise RuntimeError(f"{status_name(rc)}: {last_error()}") if rc != E_UNSUPPORTED else \
            NotImplementedError(last_error())
    try:
        t, nm, no, ws, wo, wk = (ctypes.c_void_p() for _ in range(6))
        tl, nn, nw = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        many = ctypes.c_int32()
        lib.g2n_split_get(h, ctypes.byref(t), ctypes.byref(tl), ctypes.byref(nm), ctypes.byref(no), ctypes.byref(nn),
                          ctypes.byref(ws), ctypes.byref(wo), ctypes.byref(wk), ctypes.byref(nw), ctypes.byref(many))
        text = np.frombuffer(host_bytes_at(t.value, tl.value), dtype=np.uint8)
        offs = np.ctypeslib.as_array((ctypes.c_int64 * (nn.value + 1)).from_address(no.value)).copy()
        blob = np.frombuffer(host_bytes_at(nm.value, int(offs[-1])), dtype=np.uint8)
        warns = []
        if nw.value:
            wof = np.ctypeslib.as_array((ctypes.c_int64 * (nw.value + 1)).from_address(wo.value))
            wkd = np.ctypeslib.as_array((ctypes.c_int32 * nw.value).from_address(wk.value))
            segs = host_bytes_at(ws.value, int(wof[-1]))
            warns = [(int(wkd[i]), segs[wof[i]:wof[i + 1]]) for i in range(nw.value)]
        si, ns = ctypes.c_void_p(), ctypes.c_uint64()
        lib.g2n_split_segments(h, ctypes.byref(si), ctypes.byref(ns))
        per_seg = np.ctypeslib.as_array((ctypes.c_int64 * ns.value).from_address(si.value)).copy() if ns.value \
            else np.zeros(0, dtype=np.int64)
        return text, blob, offs, warns, bool(many.value), per_seg
    finally:
        lib.g2n_split_free(h)


class GzipFailure(Exception):
    """g2n_gunzip failed: ``sub`` = gzip.py's exception kind, ``message`` its text, ``prefix``
    the bytes gzip.py's reader returned before raising."""

    def __init__(self, sub: int, message: str, prefix: bytes = b""):
        super().__init__(sub, message)
        self.sub, self.message, self.prefix = sub, message, prefix


def gunzip(data: bytes, parallel: bool = True) -> tuple[bytes, int]:
    """The library's gzip.open(...).read() (host threads); returns (bytes, member count)."""
    lib = load()
    arr = np.frombuffer(data, dtype=np.uint8)
    out, n, members, sub = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_int32(), ctypes.c_int32()
    rc = lib.g2n_gunzip(arr.ctypes.data if arr.size else None, arr.size, int(parallel), ctypes.byref(out),
                        ctypes.byref(n), ctypes.byref(members), ctypes.byref(sub))
    if rc == E_GZIP:
        msg = last_error()
        try:
            prefix = host_bytes_at(out.value, n.value) if out.value else b""
        finally:
            lib.g2n_free(out)
        raise GzipFailure(int(sub.value), msg, prefix)
    if rc != OK:
        raise RuntimeError(f"{status_name(rc)}: {last_error()}")
    try:
        return host_bytes_at(out.value, n.value), int(members.value)
    finally:
        lib.g2n_free(out)


def join_names(blob: np.ndarray, offsets: np.ndarray, sep: int = 0x0A) -> bytearray:
    """Names blob + offsets -> one bytearray, names separated by `sep` (host threads)."""
    n = len(offsets) - 1
    if n <= 0:
        return bytearray()
    out = bytearray(int(offsets[-1] - offsets[0]) + n - 1)
    if len(out):
        buf = (ctypes.c_uint8 * len(out)).from_buffer(out)
        rc = load().g2n_join_names(blob.ctypes.data, offsets.ctypes.data, n, sep, ctypes.addressof(buf))
        del buf
        if rc != OK:
            raise RuntimeError(f"{status_name(rc)}: {last_error()}")
    return out


def gather_names(blob: np.ndarray, offsets: np.ndarray, order: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """(blob, offsets) of the names in a new order: out name i = name order[i] (g2n_gather_names,
    host threads)."""
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    order = np.ascontiguousarray(order, dtype=np.int64)
    n = len(order)
    out_offs = np.zeros(n + 1, dtype=np.int64)
    if n:
        np.cumsum((offsets[1:] - offsets[:-1])[order], out=out_offs[1:])
    out = np.empty(int(out_offs[-1]), dtype=np.uint8)
    if n and len(out):
        rc = load().g2n_gather_names(blob.ctypes.data, offsets.ctypes.data, order.ctypes.data, n,
                                     out_offs.ctypes.data, out.ctypes.data)
        if rc != OK:
            raise RuntimeError(f"{status_name(rc)}: {last_error()}")
    return out, out_offs


def decimal_names(n: int, bidirected: bool = False) -> tuple[np.ndarray, np.ndarray]:
    """(blob, offsets) of the node keys of a decimal-id graph in id order (builders.py:190-198):
    node k is str(k + 1), or (bidirected) node 2j / 2j + 1 is f"{j + 1}:+" / f"{j + 1}:-" — built
    digit-width block by block with numpy, no per-name Python objects."""
    m = (n + 1) // 2 if bidirected else n
    sfx = 2 if bidirected else 0
    pieces, lens = [], []
    lo, d = 1, 1
    while lo <= m:
        hi = min(m, 10 ** d - 1)  # the d-digit values lo..hi
        v = np.arange(lo, hi + 1, dtype=np.int64)
        cols = [((v // 10 ** (d - 1 - j)) % 10 + 48).astype(np.uint8) for j in range(d)]
        if bidirected:
            w = d + 2
            rows = np.empty((len(v), 2, w), dtype=np.uint8)
            for j, c in enumerate(cols):
                rows[:, :, j] = c[:, None]
            rows[:, :, d] = ord(":")
            rows[:, 0, d + 1] = ord("+")
            rows[:, 1, d + 1] = ord("-")
            pieces.append(rows.reshape(-1))
            lens.append(np.full(2 * len(v), w, dtype=np.int64))
        else:
            pieces.append(np.stack(cols, axis=1).reshape(-1))
            lens.append(np.full(len(v), d, dtype=np.int64))
        lo, d = hi + 1, d + 1
    blob = np.concatenate(pieces) if pieces else np.zeros(0, dtype=np.uint8)
    ln = np.concatenate(lens)[:n] if lens else np.zeros(0, dtype=np.int64)
    offs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(ln, out=offs[1:])
    return blob[:int(offs[-1])], offs


def _io_error(rc: int, path: str):
    return OSError(last_error()) if rc == E_IO else RuntimeError(f"{status_name(rc)}: {last_error()}")


def write_npz(path: str, members: list[tuple[str, bytes, np.ndarray]], level: int = -1) -> None:
    """numpy savez_compressed's zip64 layout, members deflated on host threads (g2n_write_npz).
    members: (name, .npy header bytes, C-contiguous array whose raw bytes follow the header)."""
    lib = load()
    n = len(members)
    names = (ctypes.c_char_p * n)(*[m[0].encode() for m in members])
    heads_b = [m[1] for m in members]
    heads = (ctypes.c_char_p * n)(*heads_b)
    hl = (ctypes.c_uint64 * n)(*[len(h) for h in heads_b])
    arrs = [np.ascontiguousarray(m[2]) for m in members]
    datas = (ctypes.c_void_p * n)(*[a.ctypes.data if a.nbytes else None for a in arrs])
    dl = (ctypes.c_uint64 * n)(*[a.nbytes for a in arrs])
    rc = lib.g2n_write_npz(os.fsencode(path), n, names, heads, hl, datas, dl, level)
    if rc != OK:
        raise _io_error(rc, path)


def write_node_map(path: str, blob: np.ndarray, offsets: np.ndarray, check_utf8: bool) -> int:
    """save_node_map from the names blob (g2n_write_node_map); returns the first id whose name is
    not UTF-8 (only the lines before it were written), or -1."""
    lib = load()
    n = len(offsets) - 1
    bad = ctypes.c_int64(-1)
    rc = lib.g2n_write_node_map(os.fsencode(path), blob.ctypes.data if blob.size else None,
                                offsets.ctypes.data, max(n, 0), int(check_utf8), ctypes.byref(bad))
    if rc != OK:
        raise _io_error(rc, path)
    return int(bad.value)


def first_bad_utf8(blob: np.ndarray, offsets: np.ndarray) -> int:
    n = len(offsets) - 1
    if n <= 0:
        return -1
    return int(load().g2n_first_bad_utf8(blob.ctypes.data if blob.size else None, offsets.ctypes.data, n))


def device_count() -> int:
    return int(load().g2n_device_count())


def device_memory(device: int = 0) -> tuple[int, int]:
    """(free, total) HBM bytes of `device` (hipMemGetInfo, g2n_device_memory)."""
    f, t = ctypes.c_uint64(), ctypes.c_uint64()
    rc = load().g2n_device_memory(int(device), ctypes.byref(f), ctypes.byref(t))
    if rc != OK:
        raise RuntimeError(f"{status_name(rc)}: {last_error()}")
    return int(f.value), int(t.value)


def release_shared(device: int = 0) -> int:
    """Free the host entry points' cached buffers on `device` (g2n_release_shared) and, when torch is
    already loaded in this process, its allocator's unused cached blocks — HBM that only caches held:
    what an allocation that failed retries without.  Returns the library's bytes released (torch's
    count 1 when it released any)."""
    freed = ctypes.c_uint64(0)
    rc = load().g2n_release_shared(int(device), ctypes.byref(freed))
    if rc != OK:
        raise RuntimeError(f"{status_name(rc)}: {last_error()}")
    n = int(freed.value)
    torch = sys.modules.get("torch")  # (never imported here: the one-GPU path runs without torch)
    if torch is not None and torch.cuda.is_initialized():
        before = torch.cuda.memory_reserved(device)
        torch.cuda.empty_cache()
        n += 1 if torch.cuda.memory_reserved(device) < before else 0
    return n


def version() -> str:
    return load().g2n_version().decode()
