"""The chunked single-GPU build against the one-piece build on one file (wall clock, same process):
a quarter of C4 (12.5M S / 50M L, ~1.6 GB) written to the box's disk, decimal and hashed names,
chunks of 256 MiB.  Prints one JSON line per case; the matrices are compared for equality."""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from gfa2network_amd import parse_gfa, synth  # noqa: E402


def run(names):
    data = synth.host_bytes(12_500_000, 50_000_000, seed=0, names=names)
    with tempfile.NamedTemporaryFile(suffix=".gfa", delete=False, dir=os.environ.get("TMPDIR", "/tmp")) as fh:
        fh.write(data)
        path = fh.name
    del data
    try:
        out = {"names": names, "file_bytes": os.path.getsize(path)}
        parse_gfa(path, build_graph=False, build_matrix=True)  # warm: first CUDA use, file in the page cache
        parse_gfa(path, build_graph=False, build_matrix=True, chunk_bytes=256 << 20)  # warm: torch, the engine
        t = time.perf_counter()
        A = parse_gfa(path, build_graph=False, build_matrix=True)
        out["one_piece_s"] = round(time.perf_counter() - t, 3)
        t = time.perf_counter()
        C = parse_gfa(path, build_graph=False, build_matrix=True, chunk_bytes=256 << 20)
        out["chunked_256MiB_s"] = round(time.perf_counter() - t, 3)
        out["equal"] = bool(np.array_equal(A.indptr, C.indptr) and np.array_equal(A.indices, C.indices)
                            and A.data.tobytes() == C.data.tobytes())
        print(json.dumps(out), flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    for names in ("decimal", "hashed"):
        run(names)
