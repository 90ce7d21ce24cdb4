"""Synthetic GFA inputs for benchmarks and large parity tests (include/g2n_synth.h).

Deterministic and identical on host and device (gfa2network_amd/csrc/synth.h): the
host bytes feed the CPU baselines, the device bytes are bench.py's HBM-resident workload.
Named configurations follow BASELINE.json / SURVEY.md §8(d).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _native


class Spec(ctypes.Structure):
    _fields_ = [("n_segments", ctypes.c_uint64), ("n_links", ctypes.c_uint64), ("seed", ctypes.c_uint64),
                ("rc_tag", ctypes.c_int32), ("names", ctypes.c_int32), ("far_links", ctypes.c_int32)]


@dataclass(frozen=True)
class Workload:
    name: str
    n_segments: int
    n_links: int
    rc_tag: bool
    mode: dict
    note: str


# BASELINE.json configs (C1 is the DRB1 fixture file, CPU plumbing only)
WORKLOADS = {
    "C2": Workload("C2", 1_000_000, 4_000_000, False, {"directed": False},
                   "1M S / 4M L, undirected CSR"),
    "C3": Workload("C3", 1_000_000, 4_000_000, True, {"bidirected": True, "weight_tag": "RC"},
                   "1M S / 4M L + RC:i, bidirected weighted"),
    "C4": Workload("C4", 50_000_000, 200_000_000, False, {},
                   "50M S / 200M L, default (directed, MAX-SYM CSR), HBM-resident parse"),
    "C5": Workload("C5", 125_000_000, 500_000_000, False, {"directed": False},
                   "125M S / 500M L pangenome, undirected CSR (16 GB)"),
}


def _lib():
    lib = _native.load()
    if not getattr(lib, "_synth_typed", False):
        lib.g2n_synth_host.argtypes = [ctypes.POINTER(Spec), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                       ctypes.POINTER(ctypes.c_size_t)]
        lib.g2n_synth_host.restype = ctypes.c_int
        lib.g2n_synth_free_host.argtypes = [ctypes.c_void_p]
        lib.g2n_synth_device.argtypes = [ctypes.c_int, ctypes.POINTER(Spec), ctypes.POINTER(ctypes.c_void_p),
                                         ctypes.POINTER(ctypes.c_size_t)]
        lib.g2n_synth_device.restype = ctypes.c_int
        lib.g2n_synth_free_device.argtypes = [ctypes.c_void_p]
        lib.g2n_synth_download.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        lib.g2n_synth_download.restype = ctypes.c_int
        lib._synth_typed = True
    return lib


NAME_MODES = {"decimal": 0, "hashed": 1, "permuted": 2, "prefixed": 3}


def host_bytes(n_segments: int, n_links: int, seed: int = 0, rc_tag: bool = False, threads: int = 0,
               names: str = "decimal", far_links: bool = False) -> bytes:
    """The synthetic GFA as bytes, generated on the CPU.  names="hashed": segment i is named
    "s" + 8 hex digits of a bijection of i (unique, not the decimal ids "1".."N"); names="permuted":
    the decimal of a permutation of 1..N (decimal names, not in S order).  far_links: an L
    line's second segment is uniform over all segments (no id locality); names="prefixed": "s" + the
    decimal of i in S order (minigraph's s1..sN)."""
    lib = _lib()
    spec = Spec(n_segments, n_links, seed, int(rc_tag), NAME_MODES[names], int(far_links))
    ptr, n = ctypes.c_void_p(), ctypes.c_size_t()
    rc = lib.g2n_synth_host(ctypes.byref(spec), threads, ctypes.byref(ptr), ctypes.byref(n))
    if rc:
        raise RuntimeError(f"g2n_synth_host failed ({rc})")
    try:
        return _native.host_bytes_at(ptr.value, n.value)
    finally:
        lib.g2n_synth_free_host(ptr)


def write_file(path, n_segments: int, n_links: int, seed: int = 0, rc_tag: bool = False, threads: int = 0,
               names: str = "decimal", far_links: bool = False) -> int:
    """host_bytes(...) written to `path` straight from the generator's buffer (no Python bytes copy:
    a 16 GB C5 file needs 16 GB of host memory, not 32).  Returns the byte count."""
    lib = _lib()
    spec = Spec(n_segments, n_links, seed, int(rc_tag), NAME_MODES[names], int(far_links))
    ptr, n = ctypes.c_void_p(), ctypes.c_size_t()
    rc = lib.g2n_synth_host(ctypes.byref(spec), threads, ctypes.byref(ptr), ctypes.byref(n))
    if rc:
        raise RuntimeError(f"g2n_synth_host failed ({rc})")
    try:
        view = memoryview((ctypes.c_char * n.value).from_address(ptr.value)).cast("B") if n.value else b""
        with open(path, "wb") as fh:
            step = 1 << 30
            for a in range(0, n.value, step):
                fh.write(view[a:a + step])
        return n.value
    finally:
        lib.g2n_synth_free_host(ptr)


class DeviceInput:
    """Synthetic GFA generated directly in HBM; owns the device buffer."""

    def __init__(self, n_segments: int, n_links: int, seed: int = 0, rc_tag: bool = False, device: int = 0,
                 names: str = "decimal", far_links: bool = False):
        lib = _lib()
        spec = Spec(n_segments, n_links, seed, int(rc_tag), NAME_MODES[names], int(far_links))
        ptr, n = ctypes.c_void_p(), ctypes.c_size_t()
        rc = lib.g2n_synth_device(device, ctypes.byref(spec), ctypes.byref(ptr), ctypes.byref(n))
        if rc == _native.E_NOMEM and _native.release_shared(device):  # once more without the host cache
            rc = lib.g2n_synth_device(device, ctypes.byref(spec), ctypes.byref(ptr), ctypes.byref(n))
        if rc:
            raise RuntimeError(f"g2n_synth_device failed ({_native.status_name(rc)})")
        self.ptr, self.len, self.device = ptr.value, n.value, device

    def download(self) -> bytes:
        buf = np.empty(self.len, dtype=np.uint8)
        if self.len and _lib().g2n_synth_download(buf.ctypes.data, self.ptr, self.len):
            raise RuntimeError("download failed")
        return buf.tobytes()

    def free(self):
        if self.ptr:
            _lib().g2n_synth_free_device(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass
