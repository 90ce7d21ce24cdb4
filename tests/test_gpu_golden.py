"""GPU: the MI355X path reproduces every golden fixture of the real reference.

Runs the product end to end (libg2n.so through the ctypes C-ABI: read/gunzip on the host,
every parse / dictionary / triplet / CSR step on the GPU) and compares with what
sclipman/gfa2network returned for the same input, mode, weight tag and dtype: the returned
COO (stream order) or MAX-SYM CSR bit for bit, convert_format(..., "csr"), node list,
exception type + message, RuntimeWarnings and verbose strings.
"""
import numpy as np
import pytest

import golden_util as G

pytestmark = pytest.mark.gpu

ALL = list(G.combos())


def gpu_engine(name: str, g: dict):
    from gfa2network_amd import convert_format, parse_gfa

    path = str(G.input_path(name))

    def run(return_node_list, raw_bytes_id, verbose):
        return parse_gfa(path, build_graph=False, build_matrix=True, return_node_list=return_node_list,
                         raw_bytes_id=raw_bytes_id, verbose=verbose, dtype=g["dtype"],
                         weight_tag=g["weight_tag"], **g["mode"])

    return run, lambda A: convert_format(A, "csr")


@pytest.mark.parametrize("name", sorted({n for n, _ in ALL}))
def test_gpu_matches_reference(gpu, name):
    bad = []
    for n, key in ALL:
        if n != name:
            continue
        run, convert = gpu_engine(n, G.combo(n, key))
        errs = G.check(n, key, run, convert)
        if errs:
            bad.append(f"{key}: {errs[:3]}")
    assert not bad, f"{len(bad)} combos differ, e.g. {bad[:4]}"


def test_gpu_loaded_native(gpu):
    """The parity above ran through the in-tree HIP library, not anything else."""
    import gfa2network_amd._native as nat

    assert nat._lib is not None
    assert str(nat.LIB_PATH).endswith("_lib/libg2n.so")
    assert nat.device_count() >= 1
