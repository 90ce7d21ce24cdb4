"""GPU: corrupt / truncated ``.gz`` inputs behave as the reference's streaming loop does
(parser.py:108-114): the lines gzip returned before failing are parsed first — their parse
error wins, their unsupported-record warning and verbose progress come before the gzip
exception — and ``export --format edge-list`` writes their edges before raising.  Expected
outputs were produced by the reference itself (tests/golden/make_gzip_prefix_golden.py ->
tests/golden/expected/gzip_prefix.json; inputs under tests/golden/inputs_gz/), including the
cases where a malformed line is lost with the output of gzip.py's failing 8192-byte refill."""
import base64
import contextlib
import hashlib
import io
import json
import warnings
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).parent / "golden"
CASES = json.loads((GOLD / "expected" / "gzip_prefix.json").read_text())
MODES = {"default": {}, "undirected_int8": {"directed": False, "dtype": "int8"},
         "bidir_rc": {"bidirected": True, "weight_tag": "RC"}}


@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_parse_gfa_gz_prefix_matches_reference(gpu, name):
    from gfa2network_amd import parse_gfa

    case = CASES[name]
    path = GOLD / "inputs_gz" / case["file"]
    for key, want in case["parse"].items():
        mname, verbose = key.split("|")
        err = io.StringIO()
        exc = None
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            try:
                with contextlib.redirect_stderr(err), contextlib.redirect_stdout(io.StringIO()):
                    parse_gfa(str(path), build_graph=False, build_matrix=True, return_node_list=True,
                              verbose=verbose == "1", **MODES[mname])
            except Exception as e:  # noqa: BLE001
                exc = [type(e).__name__, str(e)]
        assert exc == want["exc"], key
        assert [str(x.message) for x in w if issubclass(x.category, RuntimeWarning)] == want["warnings"], key
        assert err.getvalue() == want["stderr"], key


@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_export_gz_prefix_matches_reference(gpu, name, tmp_path):
    from gfa2network_amd import export_edge_list

    case = CASES[name]
    path = GOLD / "inputs_gz" / case["file"]
    for bidir, want in case["export"].items():
        out = tmp_path / "edges.tsv"
        exc = None
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            try:
                export_edge_list(path, out, bidirected=bidir == "1")
            except Exception as e:  # noqa: BLE001
                exc = [type(e).__name__, str(e)]
        got = out.read_bytes()
        assert len(got) == want["text_len"] and hashlib.sha256(got).hexdigest() == want["text_sha256"], bidir
        if want["text_b64"] is not None:
            assert got == base64.b64decode(want["text_b64"]), bidir
        assert exc == want["exc"], bidir
        assert [str(x.message) for x in w if issubclass(x.category, RuntimeWarning)] == want["warnings"], bidir
