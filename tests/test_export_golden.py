"""export --format edge-list (cli.py:264-281): the oracle's restatement pinned against the
reference's own outputs (tests/golden/expected/export.json, made by make_export_golden.py
from the real reference), every input x {plain, --bidirected}.  CPU only."""
import base64
import gzip
import json
import warnings
from pathlib import Path

import numpy as np
import pytest

from gfa2network_amd._native import RawResult
from gfa2network_amd.api import raise_for_status

HERE = Path(__file__).resolve().parent
INPUTS = HERE / "golden" / "inputs"
EXPECTED = json.loads((HERE / "golden" / "expected" / "export.json").read_text())


def load_input(name: str) -> bytes:
    data = (INPUTS / name).read_bytes()
    return gzip.decompress(data) if name.endswith(".gz") else data


def exc_of(err):
    """The exception the reference raises for an oracle error, as [type, message]."""
    if err is None:
        return None
    kind, payload = err
    try:
        if kind == "decode":
            payload.decode()
        else:
            raise_for_status(RawResult(status=payload.status, err_detail=payload.err_detail,
                                       err_index=payload.err_index, err_value=payload.err_value),
                             np.dtype("bool"))
    except Exception as e:  # noqa: BLE001
        return [type(e).__name__, str(e)]
    raise AssertionError("no exception for an oracle error")


def expected(key):
    e = EXPECTED[key]
    return base64.b64decode(e["text_b64"]) if e["text_b64"] is not None else b"", e["exc"], e["warnings"]


@pytest.mark.parametrize("key", sorted(EXPECTED))
def test_oracle_export_matches_reference(oracle_lib, key):
    name, bidir = key.split("|")
    text, err, first = oracle_lib.export_edge_list(load_input(name), bidirected=bidir == "1")
    want_text, want_exc, want_warn = expected(key)
    assert text == want_text
    assert exc_of(err) == want_exc
    got_warn = [f"Skipping unsupported record: {chr(first.warn_byte)}"] if first.has_warning else []
    assert got_warn == want_warn


def test_export_cli_parser_flags():
    from gfa2network_amd.cli import _parser

    a = _parser().parse_args(["export", "x.gfa", "--bidirected", "--output", "o.tsv"])
    assert (a.cmd, a.format, a.bidirected, a.output) == ("export", "edge-list", True, "o.tsv")
    assert _parser().parse_args(["export", "x.gfa"]).output == "-"
