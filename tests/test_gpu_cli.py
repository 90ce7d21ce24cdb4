"""GPU: `python -m gfa2network_amd convert ... --matrix` — the reference's CLI tests
(tests/test_matrix_asym.py, test_matrix_dtype.py, test_matrix_nodes_map.py,
test_limits.py of sclipman/gfa2network) re-run against the GPU CLI, plus the written
.npz / .nodes.tsv checked against the golden arrays of the reference."""
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import scipy.sparse as sp

import golden_util as G

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
SAMPLE_GFA = b"S\ts1\t4\nS\ts2\t4\nL\ts1\t+\ts2\t-\t0M\n"


def cli(*args, check=True):
    return subprocess.run([sys.executable, "-m", "gfa2network_amd", *map(str, args)], cwd=ROOT, check=check,
                          capture_output=True, text=True)


@pytest.fixture
def sample(tmp_path):
    p = tmp_path / "sample.gfa"
    p.write_bytes(SAMPLE_GFA)
    return p


def test_matrix_asymmetric(gpu, sample, tmp_path):
    out = tmp_path / "adj.npz"
    r = cli("convert", sample, "--matrix", out, "--asymmetric")
    assert r.stdout.startswith("Using backend: networkx")
    arr = sp.load_npz(out).toarray()
    assert not (arr == arr.T).all()


def test_matrix_dtype(gpu, sample, tmp_path):
    out = tmp_path / "adj.npz"
    cli("convert", sample, "--matrix", out, "--dtype", "bool")
    assert sp.load_npz(out).dtype == bool


def test_matrix_node_map(gpu, sample, tmp_path):
    out = tmp_path / "adj.npz"
    cli("convert", sample, "--matrix", out)
    A = sp.load_npz(out)
    lines = Path(str(out) + ".nodes.tsv").read_text().strip().splitlines()
    assert len(lines) == A.shape[0]
    for i, line in enumerate(lines):
        idx, node = line.split("\t")
        assert int(idx) == i


def _big(tmp_path, n=400):
    lines = [f"S\t{i}\t*\n" for i in range(n)] + [f"L\t{i}\t+\t{i+1}\t+\t0M\n" for i in range(n - 1)]
    p = tmp_path / "big.gfa"
    p.write_text("".join(lines))
    return p


def test_dense_matrix_limit(gpu, tmp_path):
    from gfa2network_amd.cli import main

    with pytest.raises(SystemExit):  # --max-dense-gb after `convert` is an argparse error
        main(["convert", str(_big(tmp_path)), "--matrix", str(tmp_path / "dense.npy"), "--max-dense-gb", "0.001"])


def test_dense_matrix_limit_respects_dtype(gpu, tmp_path):
    from gfa2network_amd.cli import main

    out = tmp_path / "dense.npy"
    main(["--max-dense-gb", "0.001", "convert", str(_big(tmp_path)), "--matrix", str(out), "--dtype", "float32"])
    assert out.exists()


def test_dense_guard_fires(gpu, tmp_path):
    from gfa2network_amd.cli import main

    with pytest.raises(SystemExit, match="dense export would allocate"):
        main(["--max-dense-gb", "0.000001", "convert", str(_big(tmp_path)), "--matrix", str(tmp_path / "d.npy")])


@pytest.mark.parametrize("flags,key", [([], "default|-|float64"), (["--undirected"], "undirected|-|float64"),
                                       (["--asymmetric"], "asym|-|float64"),
                                       (["--bidirected", "--keep-directed-bidir"], "bidir_keep|-|float64"),
                                       (["--dtype", "bool"], "default|-|bool")])
def test_drb1_npz_matches_reference(gpu, tmp_path, flags, key):
    out = tmp_path / "drb1.npz"
    cli("convert", G.input_path("drb1"), "--matrix", out, *flags)
    A = sp.load_npz(out)
    g = G.combo("drb1", key)
    a = g["arrays"]
    assert A.format == "csr"
    for k in ("indptr", "indices", "data"):
        assert G.bits_equal(getattr(A, k), G.arr(a[f"csr/{k}"])), k
    blob = G.arr(a["names_blob"]).tobytes()
    offs = G.arr(a["names_offsets"])
    want = "".join(f"{i}\t{blob[offs[i]:offs[i+1]].decode()}\n" for i in range(len(offs) - 1))
    assert Path(str(out) + ".nodes.tsv").read_text() == want


def test_stdin_and_gzip(gpu, tmp_path):
    import gzip

    data = G.input_bytes("w")
    gz = tmp_path / "w.gfa.gz"
    gz.write_bytes(gzip.compress(data))
    out1, out2 = tmp_path / "a.npz", tmp_path / "b.npz"
    cli("convert", gz, "--matrix", out1, "--weight-tag", "RC")
    subprocess.run([sys.executable, "-m", "gfa2network_amd", "convert", "-", "--matrix", str(out2), "--weight-tag",
                    "RC"], cwd=ROOT, input=data, check=True, capture_output=True)
    A, B = sp.load_npz(out1), sp.load_npz(out2)
    assert (A != B).nnz == 0 and A.dtype == B.dtype


def test_missing_file_raises_oserror(gpu, tmp_path):
    from gfa2network_amd import parse_gfa

    with pytest.raises(FileNotFoundError):
        parse_gfa(tmp_path / "nope.gfa", build_graph=False, build_matrix=True)
    with pytest.raises(IsADirectoryError):
        parse_gfa(tmp_path, build_graph=False, build_matrix=True)
    bad = tmp_path / "bad.gfa.gz"
    bad.write_bytes(b"not gzip at all")
    import gzip

    with pytest.raises(gzip.BadGzipFile):
        parse_gfa(bad, build_graph=False, build_matrix=True)


def test_single_gpu_path_without_torch(gpu, tmp_path):
    """The single-GPU path needs no torch: with torch unimportable, parse_gfa + convert_format run
    on the GPU through libg2n.so alone and give what this (torch-importing) process gives."""
    import subprocess
    import sys

    import numpy as np

    from gfa2network_amd import convert_format, parse_gfa

    gfa = Path(__file__).parent / "golden" / "inputs" / "DRB1-3123_unsorted.gfa"
    code = (
        "import sys; sys.modules['torch'] = None\n"
        "import numpy as np\n"
        "from gfa2network_amd import convert_format, parse_gfa\n"
        f"A, nodes = parse_gfa({str(gfa)!r}, build_graph=False, build_matrix=True, return_node_list=True,"
        " directed=False)\n"
        "C = convert_format(A, 'csr')\n"
        "assert 'torch' not in sys.modules or sys.modules['torch'] is None\n"
        f"np.savez({str(tmp_path / 'out.npz')!r}, p=C.indptr, i=C.indices, d=C.data, n=np.array(nodes))\n"
    )
    r = subprocess.run([sys.executable, "-c", code], cwd=str(Path(__file__).parent.parent), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    got = np.load(tmp_path / "out.npz")
    A, nodes = parse_gfa(gfa, build_graph=False, build_matrix=True, return_node_list=True, directed=False)
    C = convert_format(A, "csr")
    assert np.array_equal(got["p"], C.indptr) and np.array_equal(got["i"], C.indices)
    assert got["d"].tobytes() == C.data.tobytes() and got["n"].tolist() == nodes
