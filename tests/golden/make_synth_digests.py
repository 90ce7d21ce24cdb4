#!/usr/bin/env python3
"""Digests of the oracle's answers on full-size BASELINE configs (tests/golden/expected/synth_digests.json).

Runs in the build container (CPU): the synthetic generator (gfa2network_amd/csrc/synth.h, host ==
device bytes) feeds oracle/g2n_oracle.cpp (the restatement pinned against the reference's
goldens); the GPU tests compare the product's arrays with these digests, so a
full-size bit-exact check on the GPU box costs one sha256 instead of a second oracle run there.

digest = sha256(int32 indptr | int32 indices | data bytes) for a CSR answer,
         sha256(int32 rows | int32 cols | data bytes) for a COO answer; names = sha256 of the
         names blob (id order) — what parse_gfa(..., return_node_list=True) and
         convert_format(A, "csr") return (builders.py:278-299, utils.py:40-63).

usage: python tests/golden/make_synth_digests.py C2 C3 C4
"""
import hashlib
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
OUT = ROOT / "tests" / "golden" / "expected" / "synth_digests.json"

CASES = {  # name -> (n_segments, n_links, rc_tag, seed, mode[, segment names])
    "C2": (1_000_000, 4_000_000, False, 0, {"directed": False}),
    "C3": (1_000_000, 4_000_000, True, 0, {"bidirected": True, "weight_tag": "RC"}),
    "C4": (50_000_000, 200_000_000, False, 0, {}),
    # C4's dimensions with the decimal names permuted (synth names="permuted"): the direct-address tier
    "C4P": (50_000_000, 200_000_000, False, 0, {}, "permuted"),
    # ... and minigraph's prefixed names "s1".."sN" in S order (synth names="prefixed"): the direct tier
    "C4X": (50_000_000, 200_000_000, False, 0, {}, "prefixed"),
}


def digest(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main(names):
    from gfa2network_amd import synth
    from oracle import oracle

    doc = json.loads(OUT.read_text()) if OUT.exists() else {}
    for name in names:
        n_s, n_l, rc, seed, mode = CASES[name][:5]
        names_mode = CASES[name][5] if len(CASES[name]) > 5 else "decimal"
        t0 = time.time()
        data = synth.host_bytes(n_s, n_l, seed=seed, rc_tag=rc, names=names_mode)
        o = oracle.run(data, **mode)
        assert o.status == 0, o.status
        ent = {"n_segments": n_s, "n_links": n_l, "rc_tag": rc, "seed": seed, "mode": mode, "dtype": "float64",
               "segment_names": names_mode,
               "input_bytes": len(data), "n_nodes": int(o.n_nodes),
               "names": digest(o.names_blob), "names_bytes": int(o.names_offsets[-1])}
        if o.maxsym:
            ent["parse"] = {"format": "csr", "nnz": int(len(o.ms_indices)),
                            "digest": digest(o.ms_indptr.astype(np.int32), o.ms_indices.astype(np.int32), o.ms_data)}
        else:
            ent["parse"] = {"format": "coo", "nnz": int(len(o.rows)),
                            "digest": digest(o.rows.astype(np.int32), o.cols.astype(np.int32), o.data)}
        ent["csr"] = {"nnz": int(len(o.sum_indices)),
                      "digest": digest(o.sum_indptr.astype(np.int32), o.sum_indices.astype(np.int32), o.sum_data)}
        ent["oracle_s"] = round(time.time() - t0, 1)
        doc[name] = ent
        print(name, json.dumps(ent), flush=True)
        del o, data
        OUT.write_text(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:] or list(CASES))
