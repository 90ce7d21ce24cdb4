"""convert_format / save_matrix verbose output against the reference's (utils.py:40-105), tqdm
branch (tqdm is importable here, as in the reference's environment): the stderr the reference
wrote for each case (tests/golden/make_verbose_golden.py -> expected/verbose.json, elapsed times
normalised) and the exception.  Conversions that need no GPU run on the CPU; the csr / csc
conversions of a COO (the GPU's coo.tocsr) run in the -m gpu variant.  Also dok: the result is
scipy's own A.asformat("dok") (utils.py:55)."""
import json
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).parent / "golden"))
from make_verbose_golden import cases, run  # noqa: E402

GOLD = json.loads((Path(__file__).parent / "golden" / "expected" / "verbose.json").read_text())


def _needs_gpu(c):
    return c["kind"] == "convert" and c["src"] == "coo" and c["arg"].lower() in ("csr", "csc")


def _check(tmp_path, gpu_cases: bool):
    from gfa2network_amd import api

    assert api._HAS_TQDM
    A, cs = cases()
    got = run(api.convert_format, api.save_matrix, tmp_path)
    assert len(got) == len(GOLD)
    n = 0
    for g, want in zip(got, GOLD):
        if _needs_gpu(want) != gpu_cases:
            continue
        assert (g["kind"], g["arg"], g["src"]) == (want["kind"], want["arg"], want["src"])
        assert g["stderr"] == want["stderr"], (want, g)
        assert g["exc"] == want["exc"], (want, g)
        n += 1
    assert n


def test_verbose_output_matches_reference_cpu(tmp_path, monkeypatch):
    # the GPU conversions are replaced by scipy's so the whole run completes without a device;
    # only the cases that never reach the GPU are compared here
    from gfa2network_amd import api

    monkeypatch.setattr(api, "_native_tocsr", lambda A, device=0: A.tocsr())
    monkeypatch.setattr(api, "_native_tocsc", lambda A, device=0: A.tocsc())
    _check(tmp_path, gpu_cases=False)


@pytest.mark.gpu
def test_verbose_output_matches_reference_gpu(gpu, tmp_path):
    _check(tmp_path, gpu_cases=True)


def test_convert_format_dok_is_scipy_asformat():
    import scipy.sparse as sp

    from gfa2network_amd import convert_format

    rng = np.random.default_rng(3)
    rows = rng.integers(0, 50, 400)
    cols = rng.integers(0, 50, 400)
    vals = rng.choice([0.1, 1e16, -1e16, 3.0, 0.0], 400)
    A = sp.coo_matrix((vals, (rows, cols)), shape=(50, 50))
    for M in (A, A.tocsr()):
        D = convert_format(M, "dok")
        W = M.asformat("dok")
        assert D.format == "dok" and D.shape == W.shape and D.dtype == W.dtype
        assert dict(D.items()) == dict(W.items())
