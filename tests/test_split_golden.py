"""parse_gfa(..., split_on_alignment=True) (builders.py:110-128 -> _parse_gfa_split,
builders.py:302-568) against fixtures the REAL reference produced
(tests/golden/make_split_golden.py -> expected/split.json: 60+ inputs x 8 flag modes; the
returned matrix bit for bit, node list, RuntimeWarnings in order, exception type + message).

CPU: the product's host logic (api._parse_gfa_split: the split mapping and rendering of
csrc/g2n_split.cpp, the warnings, the bidirected id shift) with the ORACLE as the build engine
(the checker stands in for the GPU build only).  GPU: the product end to end (the GPU parse,
the native split render, the GPU build of the rendered stream)."""
from __future__ import annotations

import base64
import json
import warnings
from pathlib import Path

import numpy as np
import pytest

HERE = Path(__file__).resolve().parent / "golden"
DATA = json.loads((HERE / "expected" / "split.json").read_text())
MODES, CASES = DATA["modes"], DATA["cases"]
KEYS = sorted(CASES)


def _check(key: str, call) -> None:
    exp = CASES[key]
    with warnings.catch_warnings(record=True) as ws:
        warnings.simplefilter("always")
        try:
            A, nodes = call()
            exc = None
        except Exception as e:  # noqa: BLE001 - compared as data
            exc = [type(e).__name__, str(e)]
    got_w = [[w.category.__name__, str(w.message)] for w in ws]
    assert exc == exp["exc"], key
    assert got_w == exp["warnings"], key
    if exc is not None:
        return
    assert A.format == exp["format"] and list(A.shape) == exp["shape"] and str(A.dtype) == exp["dtype"], key
    arrs = {"indptr": A.indptr, "indices": A.indices} if A.format == "csr" else {"row": A.row, "col": A.col}
    arrs["data"] = A.data
    for name, (dt, b64) in exp["arrays"].items():
        assert str(arrs[name].dtype) == dt, (key, name)
        assert np.ascontiguousarray(arrs[name]).tobytes() == base64.b64decode(b64), (key, name)
    want = [base64.b64decode(x) for x in exp["nodes"]]
    got = [x if isinstance(x, bytes) else x.encode() for x in nodes]
    assert got == want, key
    assert (bool(nodes) and isinstance(nodes[0], bytes)) == exp["nodes_bytes"], key


def _oracle_build(oracle_lib):
    from oracle import oracle

    def build(src, mode, want_names):
        assert not isinstance(src, str), "golden inputs are clean: the bytes are always in hand"
        return oracle.to_raw(oracle.run(bytes(src), **mode), "parse")

    return build


@pytest.mark.parametrize("key", KEYS)
def test_split_host_logic_with_oracle_engine(oracle_lib, key):
    from gfa2network_amd.api import _parse_gfa_split

    path, mode = key.split("|")
    kw = dict(MODES[mode])
    kw.setdefault("directed", True)
    _check(key, lambda: _parse_gfa_split(
        str(HERE / path), build_matrix=True, directed=kw.get("directed", True), weight_tag=kw.get("weight_tag"),
        strip_orientation=kw.get("strip_orientation", False), bidirected=kw.get("bidirected", False),
        keep_directed_bidir=kw.get("keep_directed_bidir", False), dtype=kw.get("dtype", "float64"),
        asymmetric=kw.get("asymmetric", False), raw_bytes_id=kw.get("raw_bytes_id", False), return_node_list=True,
        device=0, build=_oracle_build(oracle_lib)))


def test_split_render_text_shapes():
    from gfa2network_amd import _native

    text, blob, offs, warns, many, _ = _native.split_render(
        b"S\ta\t10\t*\nS\tb\t4\t*\nE\te\ta+\t2\t6\tb-\t0\t4\t*\tRC:i:3\nL\ta\t+\tq\t-\t0M\n", False)
    names = [bytes(blob[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)]
    assert names == [b"a:0-2", b"a:2-6", b"a:6-10", b"b:0-4"]
    assert bytes(text).splitlines() == [
        b"S\ta:0-2", b"S\ta:2-6", b"S\ta:6-10", b"E\t*\ta:0-2\t+\ta:2-6\t+", b"E\t*\ta:2-6\t+\ta:6-10\t+",
        b"S\tb:0-4", b"E\t*\ta:2-6\t+\tb:0-4\t-\tRC:i:3"]
    assert warns == [(1, b"q")] and not many
    # a coordinate beyond int64 is outside this implementation (Python ints are unbounded)
    with pytest.raises(NotImplementedError):
        _native.split_render(b"S\ta\t99999999999999999999\t*\n", False)


@pytest.mark.gpu
@pytest.mark.parametrize("key", KEYS)
def test_split_gpu_equals_reference(gpu, key):
    from gfa2network_amd import parse_gfa

    path, mode = key.split("|")
    _check(key, lambda: parse_gfa(str(HERE / path), build_graph=False, build_matrix=True, return_node_list=True,
                                  split_on_alignment=True, **MODES[mode]))


@pytest.mark.gpu
def test_split_gpu_file_object_and_build_matrix_false(gpu):
    import io

    from gfa2network_amd import parse_gfa

    key = "inputs_split/e_coords.gfa|bidir"
    data = (HERE / "inputs_split" / "e_coords.gfa").read_bytes()
    _check(key, lambda: parse_gfa(io.BytesIO(data), build_graph=False, build_matrix=True, return_node_list=True,
                                  split_on_alignment=True, **MODES["bidir"]))
    # builders.py:563-568: neither output requested -> None (after the parse and the warnings)
    assert parse_gfa(io.BytesIO(data), build_graph=False, build_matrix=False, split_on_alignment=True) is None


@pytest.mark.gpu
@pytest.mark.parametrize("name,mode,flags", [("e_coords", "default", []), ("c_records", "bidir", ["--bidirected"]),
                                            ("many_nodes", "asym", ["--asymmetric"])])
def test_split_cli_convert(gpu, tmp_path, name, mode, flags):
    """`convert --split-on-alignment --matrix x.npz` (cli.py:111-115, 193-250): the .npz holds
    convert_format(A, "csr") of the reference's split matrix, the sidecar its node list."""
    import subprocess
    import sys

    import scipy.sparse as sp

    out = tmp_path / "x.npz"
    subprocess.run([sys.executable, "-m", "gfa2network_amd", "convert", str(HERE / "inputs_split" / f"{name}.gfa"),
                    "--matrix", str(out), "--split-on-alignment", *flags], check=True, capture_output=True,
                   cwd=Path(__file__).resolve().parents[1])
    exp = CASES[f"inputs_split/{name}.gfa|{mode}"]
    arr = {k: np.frombuffer(base64.b64decode(b), dtype=dt) for k, (dt, b) in exp["arrays"].items()}
    n = exp["shape"][0]
    if exp["format"] == "csr":
        want = sp.csr_matrix((arr["data"], arr["indices"], arr["indptr"]), shape=(n, n))
    else:
        want = sp.coo_matrix((arr["data"], (arr["row"], arr["col"])), shape=(n, n)).tocsr()
    A = sp.load_npz(out)
    assert A.format == "csr"
    for k in ("indptr", "indices", "data"):
        assert np.array_equal(getattr(A, k), getattr(want, k)), k
    names = [base64.b64decode(x).decode() for x in exp["nodes"]]
    assert Path(str(out) + ".nodes.tsv").read_text() == "".join(f"{i}\t{v}\n" for i, v in enumerate(names))


@pytest.mark.gpu
def test_split_gpu_gzip_and_stdin(gpu, tmp_path):
    """The split path reads its input by the reference's source rules (parser.py:100-112): a .gz
    by name (gzip.open), '-' as stdin; the result equals the plain file's golden."""
    import gzip
    import subprocess
    import sys

    key = "inputs_split/missing_segments.gfa|undirected"
    data = (HERE / "inputs_split" / "missing_segments.gfa").read_bytes()
    gz = tmp_path / "m.gfa.gz"
    gz.write_bytes(gzip.compress(data))
    from gfa2network_amd import parse_gfa

    _check(key, lambda: parse_gfa(str(gz), build_graph=False, build_matrix=True, return_node_list=True,
                                  split_on_alignment=True, **MODES["undirected"]))
    code = ("import sys, json; sys.path.insert(0, %r); from gfa2network_amd import parse_gfa; "
            "A, n = parse_gfa('-', build_graph=False, build_matrix=True, return_node_list=True, "
            "split_on_alignment=True, directed=False); A = A.tocoo(); "
            "print(json.dumps([list(A.shape), A.row.tolist(), A.col.tolist(), A.data.tolist(), n]))"
            % str(Path(__file__).resolve().parents[1]))
    out = subprocess.run([sys.executable, "-W", "ignore", "-c", code], input=data, capture_output=True, check=True)
    shape, rows, cols, vals, nodes = json.loads(out.stdout.decode().strip().splitlines()[-1])
    exp = CASES[key]
    assert shape == exp["shape"]
    assert rows == np.frombuffer(base64.b64decode(exp["arrays"]["row"][1]), dtype=exp["arrays"]["row"][0]).tolist()
    assert cols == np.frombuffer(base64.b64decode(exp["arrays"]["col"][1]), dtype=exp["arrays"]["col"][0]).tolist()
    assert vals == np.frombuffer(base64.b64decode(exp["arrays"]["data"][1]), dtype=exp["arrays"]["data"][0]).tolist()
    assert [x.encode() for x in nodes] == [base64.b64decode(x) for x in exp["nodes"]]


@pytest.mark.gpu
def test_split_gpu_corrupt_gzip_raises_like_plain_path(gpu, tmp_path):
    """A truncated .gz: the split path raises what the plain parse raises (gzip.py's EOFError
    after the whole lines before it were parsed)."""
    import gzip

    from gfa2network_amd import parse_gfa

    data = (HERE / "inputs_split" / "e_coords.gfa").read_bytes() * 50
    gz = tmp_path / "t.gfa.gz"
    gz.write_bytes(gzip.compress(data)[:-20])
    kw = dict(build_graph=False, build_matrix=True, return_node_list=True)
    with pytest.raises(EOFError) as plain:
        parse_gfa(str(gz), **kw)
    with pytest.raises(EOFError) as split:
        parse_gfa(str(gz), split_on_alignment=True, **kw)
    assert str(plain.value) == str(split.value)
