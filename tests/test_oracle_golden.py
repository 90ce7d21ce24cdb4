"""CPU: the oracle (C++ restatement) + the product's host-side finalize() reproduce every
golden fixture the real reference produced (tests/golden/make_golden.py).

This pins the oracle before it is trusted as the GPU path's checker, and exercises the
shim's Python-object assembly, warnings, exceptions and verbose strings on the CPU.
"""
import numpy as np
import pytest
import scipy.sparse as sp

import golden_util as G
from gfa2network_amd.api import finalize

MODE_KEYS = ("directed", "bidirected", "keep_directed_bidir", "asymmetric", "strip_orientation")


def oracle_engine(oracle_mod, data: bytes, g: dict):
    mode = g["mode"]
    dt = np.dtype(g["dtype"])

    def run(return_node_list, raw_bytes_id, verbose):
        o = oracle_mod.run(data, dtype=dt, weight_tag=g["weight_tag"], **{k: mode[k] for k in mode})
        raw = oracle_mod.to_raw(o, "parse")
        return finalize(raw, dtype=dt, return_node_list=return_node_list, raw_bytes_id=raw_bytes_id,
                        verbose=verbose)

    def convert(A):
        if A.format == "csr":
            return A
        o = oracle_mod.run(data, dtype=dt, weight_tag=g["weight_tag"], **{k: mode[k] for k in mode})
        raw = oracle_mod.to_raw(o, "csr")
        return sp.csr_matrix((raw.data, raw.indices, raw.indptr), shape=A.shape, dtype=dt)

    return run, convert


ALL = list(G.combos())


@pytest.mark.parametrize("name", sorted({n for n, _ in ALL}))
def test_oracle_matches_reference(oracle_lib, name):
    data = G.input_bytes(name)
    bad = []
    for n, key in ALL:
        if n != name:
            continue
        run, convert = oracle_engine(oracle_lib, data, G.combo(n, key))
        errs = G.check(n, key, run, convert)
        if errs:
            bad.append(f"{key}: {errs[:3]}")
    assert not bad, f"{len(bad)} combos differ, e.g. {bad[:5]}"
