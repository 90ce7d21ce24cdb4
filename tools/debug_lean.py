"""Debug: the tile-local lean parse (k_tile_lean) against the other paths on a small decimal GFA."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_gpu_diff import _decimal_gfa  # noqa: E402

from gfa2network_amd import _native as nat  # noqa: E402

data = "".join(_decimal_gfa(4, 400, 2400)).encode()
print("bytes", len(data))
out = {}
for name, flag in (("default", 0), ("nogroup", nat.TEST_NO_GROUP), ("notile", nat.TEST_NO_TILE_LOCAL)):
    for mode in ({}, {"directed": False}):
        o = nat.make_options(dtype="int32", output=nat.OUT_CSR, **mode)
        o.reserved[1] = flag
        r = nat.build_from_buffer(data, o)
        key = (name, str(mode))
        out[key] = r
        print(key, r.status, r.n_nodes, r.nnz, sorted(r.phase_ms))
for mode in ({}, {"directed": False}):
    a = out[("notile", str(mode))]
    for name in ("default", "nogroup"):
        b = out[(name, str(mode))]
        for f in ("indptr", "indices", "data"):
            x, y = np.asarray(getattr(a, f)), np.asarray(getattr(b, f))
            if x.shape != y.shape or not np.array_equal(x, y):
                d = np.flatnonzero(x[:min(len(x), len(y))] != y[:min(len(x), len(y))])
                print("DIFF", name, mode, f, x.shape, y.shape, d[:5], x[d[:5]] if len(d) else None,
                      y[d[:5]] if len(d) else None)
print("done")
