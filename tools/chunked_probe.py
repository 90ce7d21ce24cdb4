"""The chunked single-GPU build against the one-piece build on one file (wall clock, same process):
a quarter of C4 (12.5M S / 50M L, ~1.6 GB) written to the box's disk, decimal and hashed names,
chunks of 256 MiB (argv: other sizes in MiB).  Prints one JSON line per case; the matrices are
compared for equality."""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from gfa2network_amd import parse_gfa, synth  # noqa: E402


def run(names, chunk_mib):
    data = synth.host_bytes(12_500_000, 50_000_000, seed=0, names=names)
    with tempfile.NamedTemporaryFile(suffix=".gfa", delete=False, dir=os.environ.get("TMPDIR", "/tmp")) as fh:
        fh.write(data)
        path = fh.name
    del data
    try:
        out = {"names": names, "file_bytes": os.path.getsize(path)}
        parse_gfa(path, build_graph=False, build_matrix=True)  # warm: first CUDA use, file in the page cache
        parse_gfa(path, build_graph=False, build_matrix=True, chunk_bytes=chunk_mib[0] << 20)  # warm: torch, engine
        t = time.perf_counter()
        A = parse_gfa(path, build_graph=False, build_matrix=True)
        out["one_piece_s"] = round(time.perf_counter() - t, 3)
        for mib in chunk_mib:
            t = time.perf_counter()
            C = parse_gfa(path, build_graph=False, build_matrix=True, chunk_bytes=mib << 20)
            out[f"chunked_{mib}MiB_s"] = round(time.perf_counter() - t, 3)
            out[f"equal_{mib}"] = bool(np.array_equal(A.indptr, C.indptr) and np.array_equal(A.indices, C.indices)
                                       and A.data.tobytes() == C.data.tobytes())
        print(json.dumps(out), flush=True)
    finally:
        os.unlink(path)


def stages(names, mib):
    """The chunked general / decimal build's own stage timings (ShardResult.timings_ms) for one size."""
    import torch

    from gfa2network_amd import shard

    torch.zeros(1, device="cuda")  # torch's HIP context first (as parse_gfa's callers have it)
    data = synth.host_bytes(12_500_000, 50_000_000, seed=0, names=names)
    eng = shard.HipEngine(0)
    try:
        src = shard.HostSource(np.frombuffer(data, dtype=np.uint8))
        shard.build_chunked(src, engine=eng, chunk_bytes=mib << 20)  # warm
        t = time.perf_counter()
        r = shard.build_chunked(src, engine=eng, chunk_bytes=mib << 20)
        wall = round(time.perf_counter() - t, 3)
        print(json.dumps({"names": names, "chunk_mib": mib, "wall_s": wall, "path": r.parse_path,
                          "timings_ms": {k: round(v, 1) for k, v in r.timings_ms.items()}}), flush=True)
    finally:
        eng.close()


if __name__ == "__main__":
    if sys.argv[1:2] == ["stages"]:  # tools/chunked_probe.py stages <MiB> ...: the stage timings
        for mib in [int(x) for x in sys.argv[2:]] or [256]:
            stages("hashed", mib)
        sys.exit(0)
    sizes = [int(x) for x in sys.argv[1:]] or [256]
    for names in ("decimal", "hashed"):
        run(names, sizes)
