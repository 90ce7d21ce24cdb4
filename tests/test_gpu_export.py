"""GPU: export --format edge-list (cli.py:264-281) rendered in HBM (G2N_OUT_EDGE_LIST),
checked byte for byte against the reference's own outputs (tests/golden/expected/export.json:
written bytes, exception, warnings, every input x {plain, --bidirected}), the reference's
tests/test_export_edge_list.py re-run on the GPU CLI, and the oracle's restatement on a
synthetic 200k-edge input."""
import subprocess
import sys
import warnings
from pathlib import Path

import pytest

from test_export_golden import EXPECTED, INPUTS, expected

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.parametrize("key", sorted(EXPECTED))
def test_gpu_export_matches_reference(gpu, key, tmp_path):
    from gfa2network_amd import export_edge_list

    name, bidir = key.split("|")
    out = tmp_path / "edges.tsv"
    exc = None
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        try:
            export_edge_list(INPUTS / name, out, bidirected=bidir == "1")
        except Exception as e:  # noqa: BLE001
            exc = [type(e).__name__, str(e)]
    want_text, want_exc, want_warn = expected(key)
    assert out.read_bytes() == want_text
    assert exc == want_exc
    assert [str(x.message) for x in w if issubclass(x.category, RuntimeWarning)] == want_warn


def test_gpu_export_cli(gpu, tmp_path):  # the reference's tests/test_export_edge_list.py
    gfa = tmp_path / "e.gfa"
    gfa.write_bytes(b"S\ts1\t4\nS\ts2\t4\nL\ts1\t+\ts2\t+\t0M\n")
    out = tmp_path / "edges.tsv"
    subprocess.run([sys.executable, "-m", "gfa2network_amd", "export", str(gfa), "--format", "edge-list",
                    "--output", str(out)], check=True, cwd=ROOT)
    assert out.read_text().strip() == "s1\ts2"
    r = subprocess.run([sys.executable, "-m", "gfa2network_amd", "export", str(gfa), "--bidirected"], check=True,
                       cwd=ROOT, capture_output=True)
    assert r.stdout == b"s1:+\ts2:+\n"


@pytest.mark.parametrize("bidir", [False, True])
def test_gpu_export_synthetic_vs_oracle(gpu, oracle_lib, tmp_path, bidir):
    from gfa2network_amd import export_edge_list, synth

    data = synth.host_bytes(50_000, 200_000, seed=7)
    src = tmp_path / "s.gfa"
    src.write_bytes(data)
    out = tmp_path / "edges.tsv"
    export_edge_list(src, out, bidirected=bidir)
    text, err, _ = oracle_lib.export_edge_list(data, bidirected=bidir)
    assert err is None
    assert out.read_bytes() == text
    assert text.count(b"\n") == 200_000


def test_gpu_export_long_names_vs_oracle(gpu, oracle_lib, tmp_path):
    """Lines longer than the LDS stage holds per block (direct-to-HBM rendering), mixed with
    short ones, ragged block ends."""
    from gfa2network_amd import export_edge_list

    rng = __import__("random").Random(3)
    names = [("n%d_" % i + "x" * rng.choice([0, 1, 40, 300])).encode() for i in range(3000)]
    lines = [b"S\t" + nm + b"\t*\n" for nm in names]
    for _ in range(5003):
        u, v = rng.choice(names), rng.choice(names)
        lines.append(b"L\t" + u + b"\t" + rng.choice([b"+", b"-"]) + b"\t" + v + b"\t+\t0M\n")
    data = b"".join(lines)
    src = tmp_path / "long.gfa"
    src.write_bytes(data)
    for bidir in (False, True):
        out = tmp_path / "edges.tsv"
        export_edge_list(src, out, bidirected=bidir)
        text, err, _ = oracle_lib.export_edge_list(data, bidirected=bidir)
        assert err is None
        assert out.read_bytes() == text


@pytest.mark.parametrize("name", ["warn_then_error.gfa", "short_l.gfa", "bad_utf8_name.gfa", "sample.gfa"])
def test_gpu_export_gzip_and_stdin(gpu, tmp_path, name):
    """The same reference outputs through a .gz input (a parse error re-inflates the input to
    render its prefix) and through stdin (`-`, parser.py:104-105) on the CLI."""
    import gzip as gz

    from gfa2network_amd import export_edge_list

    want_text, want_exc, _ = expected(f"{name}|0")
    src = tmp_path / (name + ".gz")
    src.write_bytes(gz.compress((INPUTS / name).read_bytes()))
    out = tmp_path / "edges.tsv"
    exc = None
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        try:
            export_edge_list(src, out)
        except Exception as e:  # noqa: BLE001
            exc = [type(e).__name__, str(e)]
    assert out.read_bytes() == want_text
    assert exc == want_exc
    r = subprocess.run([sys.executable, "-m", "gfa2network_amd", "export", "-"], cwd=ROOT, capture_output=True,
                       input=(INPUTS / name).read_bytes())
    assert r.stdout == want_text
    assert (r.returncode != 0) == (want_exc is not None)
    if want_exc:
        assert r.stderr.decode().rstrip().splitlines()[-1] == f"{want_exc[0]}: {want_exc[1]}"


def _dec_cases():
    """Decimal-id inputs (S line k names "k+1", S lines first): the arithmetic render; and inputs
    that break the premise (blob render)."""
    from gfa2network_amd import synth

    base = synth.host_bytes(3000, 12_345, seed=11)  # ragged: 12345 edges, not a multiple of 4 / 1024
    lines = base.split(b"\n")
    n_s = sum(1 for ln in lines if ln.startswith(b"S"))
    yield "synthetic", base, True
    yield "one_edge", b"S\t1\t*\nS\t2\t*\nL\t1\t+\t2\t-\t0M\n", True
    yield "no_edges", b"S\t1\t*\nS\t2\t*\n", True
    yield "multi_digit", b"".join(b"S\t%d\t*\n" % k for k in range(1, 12)) + b"L\t11\t+\t9\t-\t0M\n" * 5, True
    yield "edge_before_s", b"L\t5\t+\t2\t-\t0M\n" + base, False  # first touch "5": id 0
    yield "named", base.replace(b"S\t1\t", b"S\tx\t", 1), False
    # a malformed line: the lines before it are written (the prefix takes the arithmetic render)
    yield "malformed_prefix", b"\n".join(lines[: n_s + 700] + [b"L\t1\t+"] + lines[n_s + 700:]), True


@pytest.mark.parametrize("case", ["synthetic", "one_edge", "no_edges", "multi_digit", "edge_before_s", "named",
                                  "malformed_prefix"])
def test_gpu_export_decimal_render(gpu, oracle_lib, monkeypatch, case):
    """A decimal-id build's lines are rendered from the ids (k_edge_dec_sum / k_edge_dec_text: no
    names blob); same bytes and failure as the blob render (TEST_NO_DEC_TEXT) and the oracle."""
    from gfa2network_amd import _native as nat

    data, dec = next((d, e) for n, d, e in _dec_cases() if n == case)
    for bidir in (False, True):
        opts = nat.make_options(bidirected=bidir, output=nat.OUT_EDGE_LIST)
        raw = nat.build_from_buffer(data, opts)
        text = bytes(raw.data) if raw.format == "text" else b""
        if raw.status == 0:
            assert ("names" not in raw.phase_ms) == dec, (case, sorted(raw.phase_ms))
        # the blob render forced through this call's own options (a flag set after
        # make_options never reached the build)
        ref = nat.build_from_buffer(data, nat.make_options(bidirected=bidir, output=nat.OUT_EDGE_LIST,
                                                           test_flags=nat.TEST_NO_DEC_TEXT))
        assert (raw.status, raw.err_line) == (ref.status, ref.err_line), case
        if ref.status == 0:
            assert "names" in ref.phase_ms, (case, sorted(ref.phase_ms))  # the blob path ran
        assert text == (bytes(ref.data) if ref.format == "text" else b""), (case, bidir)
        want, err, _ = oracle_lib.export_edge_list(data, bidirected=bidir)
        assert text == want, (case, bidir)
        assert (err is None) == (raw.status == 0), (case, err)
