"""Where the chunked build's time goes (diagnostics): shard.build_chunked on a quarter-C4 file with
per-stage host times, decimal names, 256 MiB chunks."""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gfa2network_amd import shard, synth  # noqa: E402

data = synth.host_bytes(12_500_000, 50_000_000, seed=0, names=sys.argv[1] if len(sys.argv) > 1 else "decimal")
with tempfile.NamedTemporaryFile(suffix=".gfa", delete=False, dir="/tmp") as fh:
    fh.write(data)
    path = fh.name
del data
eng = shard.HipEngine(0)
orig = eng.build_decimal_range


def timed(*a, **k):
    t = time.perf_counter()
    r = orig(*a, **k)
    eng.torch.cuda.synchronize()
    print("chunk", round((time.perf_counter() - t) * 1e3, 1), "ms", None if r is None else r[1], flush=True)
    return r


eng.build_decimal_range = timed
for rep in range(2):
    t = time.perf_counter()
    res = shard.build_chunked(path, engine=eng, chunk_bytes=256 << 20)
    print(json.dumps({"total_s": round(time.perf_counter() - t, 3), "path": res.parse_path, "tm": res.timings_ms}),
          flush=True)
os.unlink(path)
