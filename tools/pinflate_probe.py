"""Probe: chunk-parallel single-member inflate (g2n_pinflate.cpp) on a synthetic GFA.

    python tools/pinflate_probe.py [n_segments] [n_links]

Writes the text as ONE gzip member (bench.write_gz_single, pigz layout), then times
g2n_gunzip_chunked (phase trace with G2N_PINFLATE_TRACE=1), the member-chain reader on the same
file, and single-thread zlib on a slice.  Prints one JSON line."""
import json
import os
import sys
import tempfile
import time
import zlib
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from gfa2network_amd import _native, synth  # noqa: E402

n_s = int(sys.argv[1]) if len(sys.argv) > 1 else 16_000_000
n_l = int(sys.argv[2]) if len(sys.argv) > 2 else 64_000_000
threads = int(os.environ.get("G2N_HOST_THREADS", "16"))
data = synth.host_bytes(n_s, n_l, seed=0, threads=threads)
out = {"input_bytes": len(data), "threads": threads}
with tempfile.NamedTemporaryFile(suffix=".gz", dir=os.environ.get("TMPDIR") or "/tmp") as fh:
    t = time.perf_counter()
    out["gz_bytes"] = bench.write_gz_single(data, fh.name, threads=threads)
    out["write_s"] = round(time.perf_counter() - t, 2)
    blob = Path(fh.name).read_bytes()
_native.load()
for it in range(3):
    t = time.perf_counter()
    got = _native.gunzip_chunked(blob)
    dt = time.perf_counter() - t
assert got is not None and got[0] == data
out["chunked_s"] = round(dt, 3)
out["chunked_gbs"] = round(len(data) / dt / 1e9, 2)
out["chunks"] = got[1]
del got
t = time.perf_counter()
full, members = _native.gunzip(blob)
out["gunzip_path_s"] = round(time.perf_counter() - t, 3)
assert full == data and members == 1
del full
d = zlib.decompressobj(31)
t = time.perf_counter()
part = d.decompress(blob[: len(blob) // 8])
dt = time.perf_counter() - t
out["zlib_1thread_gbs"] = round(len(part) / dt / 1e9, 3)
print(json.dumps(out))
