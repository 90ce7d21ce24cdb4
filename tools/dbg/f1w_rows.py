"""Diagnostics: rows where the weighted SUM CSR differs from the oracle (row length, first diff)."""
import sys

import numpy as np

sys.path.insert(0, ".")
from gfa2network_amd import _native as nat  # noqa: E402
from gfa2network_amd import synth  # noqa: E402
from oracle import oracle  # noqa: E402

oracle.build()
lib = oracle
data = synth.host_bytes(200_000, 800_000, seed=7, rc_tag=True)
for mode in ({"directed": False}, {"bidirected": True}):
    raw = nat.build_from_buffer(data, nat.make_options(output=nat.OUT_CSR, dtype="float64", weight_tag="RC", **mode))
    o = lib.run(data, dtype="float64", weight_tag="RC", **mode)
    R = lib.to_raw(o, "csr")
    ip, ri = np.asarray(raw.indptr), np.asarray(R.indptr)
    print(mode, "nnz", int(ip[-1]), int(ri[-1]), "indptr equal", np.array_equal(ip, ri), flush=True)
    n = len(ri) - 1
    bad = 0
    lens = []
    for r in range(n):
        a0, a1, b0, b1 = int(ip[r]), int(ip[r + 1]), int(ri[r]), int(ri[r + 1])
        ca, cb = np.asarray(raw.indices[a0:a1]), np.asarray(R.indices[b0:b1])
        va, vb = np.asarray(raw.data[a0:a1]), np.asarray(R.data[b0:b1])
        if a1 - a0 != b1 - b0 or not np.array_equal(ca, cb) or va.tobytes() != vb.tobytes():
            bad += 1
            lens.append(b1 - b0)
            if bad <= 5:
                print(" row", r, "len", a1 - a0, b1 - b0, "cols", ca[:8], cb[:8], "vals", va[:8], vb[:8], flush=True)
    print(" bad rows", bad, "len hist", np.bincount(np.minimum(np.asarray(lens, dtype=np.int64), 80))[:81] if lens else [],
          flush=True)
