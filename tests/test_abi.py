"""CPU: the C-ABI library builds/loads and exports every symbol include/g2n.h declares;
the product path fails loudly (no CPU fallback) when no GPU is visible."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def declared_functions() -> list[str]:
    names = []
    for h in (ROOT / "include").glob("*.h"):
        text = h.read_text()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names += re.findall(r"\b(g2n_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    from gfa2network_amd import _native

    lib = _native.load()
    decl = declared_functions()
    assert decl, "no declarations found"
    missing = [n for n in decl if not hasattr(lib, n)]
    assert not missing, missing
    assert set(_native.EXPORTED) <= set(decl)


def test_abi_version_and_defaults():
    from gfa2network_amd import _native

    assert _native.load().g2n_abi_version() == _native.ABI_VERSION
    o = _native.make_options()
    assert (o.directed, o.bidirected, o.keep_directed_bidir, o.asymmetric, o.strip_orientation) == (1, 0, 0, 0, 0)
    assert o.dtype == _native.DTYPE_CODES["float64"] and o.want_node_names == 1


def test_struct_sizes_match_header(tmp_path):
    """ctypes layouts agree with the C structs: every field's offset and both sizes, as gcc lays
    out include/g2n.h."""
    import subprocess

    from gfa2network_amd import _native

    structs = {"g2n_options": _native.Options, "g2n_result": _native.Result}
    lines = []
    for cname, py in structs.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            lines.append(f'printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    src = tmp_path / "layout.c"
    src.write_text("#include <stddef.h>\n#include <stdio.h>\n#include \"g2n.h\"\nint main(void) {\n"
                   + "\n".join(lines) + "\nreturn 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), "-o", str(exe), str(src)], check=True)
    got = {}
    for ln in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        s, f, v = ln.split()
        got[(s, f)] = int(v)
    for cname, py in structs.items():
        assert got[(cname, "sizeof")] == ctypes.sizeof(py), cname
        for f in py._fields_:
            assert got[(cname, f[0])] == getattr(py, f[0]).offset, (cname, f[0])


@pytest.mark.skipif(__import__("gfa2network_amd._native", fromlist=["x"]).device_count() > 0,
                    reason="a GPU is visible")
def test_no_gpu_fails_loudly(tmp_path):
    from gfa2network_amd import parse_gfa

    p = tmp_path / "a.gfa"
    p.write_bytes(b"S\ta\nL\ta\t+\tb\t+\t*\n")
    with pytest.raises(RuntimeError, match="G2N_E_DEVICE"):
        parse_gfa(p, build_graph=False, build_matrix=True)


def test_out_of_scope_options_raise(tmp_path):
    from gfa2network_amd import parse_gfa

    p = tmp_path / "a.gfa"
    p.write_bytes(b"S\ta\n")
    with pytest.raises(NotImplementedError):
        parse_gfa(p, build_graph=True, build_matrix=False)
    with pytest.raises(NotImplementedError):
        parse_gfa(p, build_graph=False, build_matrix=True, backend="igraph")
    with pytest.raises(ValueError, match="return_node_list requires build_matrix=True"):
        parse_gfa(p, build_graph=False, build_matrix=False, return_node_list=True)
    with pytest.raises(NotImplementedError):  # another dtype with weights (unit values: test_unit_dtypes.py)
        parse_gfa(p, build_graph=False, build_matrix=True, dtype="int64", weight_tag="RC")


def test_join_names_matches_python():
    """g2n_join_names (the node list's one-pass join, api._node_list) == b"\\n".join(names)."""
    import random

    import numpy as np

    from gfa2network_amd import _native

    r = random.Random(3)
    for n in (1, 2, 7, 70_000, 200_001):
        names = [bytes(r.randrange(256) for _ in range(r.choice([0, 1, 3, 9]))).replace(b"\n", b"x")
                 for _ in range(n)]
        offs = np.zeros(n + 1, dtype=np.int64)
        offs[1:] = np.cumsum([len(x) for x in names])
        blob = np.frombuffer(b"".join(names) or b"\0", dtype=np.uint8)
        assert bytes(_native.join_names(blob, offs)) == b"\n".join(names)


def test_library_loads_without_importing_torch():
    """libg2n.so loads without `import torch` (torch's bundled HIP runtime is preloaded by path
    when torch is installed), and loads with torch not importable at all."""
    import subprocess
    import sys
    from pathlib import Path

    root = str(Path(__file__).resolve().parent.parent)
    for pre in ("", "sys.modules['torch'] = None\n"):
        code = ("import sys\n" + pre + "from gfa2network_amd import _native, parse_gfa\n_native.load()\n"
                "assert sys.modules.get('torch') is None, 'torch was imported'\nprint(_native.version())\n")
        r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        assert "gfa2network-amd" in r.stdout


def test_library_version_matches_package():
    import gfa2network_amd
    from gfa2network_amd import _native

    assert _native.version() == f"gfa2network-amd {gfa2network_amd.__version__} (gfx950)"


def test_synthetic_far_links_mode():
    """The benchmark generator's far_links mode (include/g2n_synth.h): the same S lines and L sources,
    the second segment uniform over all segments instead of a few ids after the source."""
    from gfa2network_amd import synth

    near = synth.host_bytes(1000, 5000, seed=3).decode().splitlines()
    far = synth.host_bytes(1000, 5000, seed=3, far_links=True).decode().splitlines()
    assert [x for x in near if x[0] != "L"] == [x for x in far if x[0] != "L"]
    ln = [x.split("\t") for x in near if x[0] == "L"]
    lf = [x.split("\t") for x in far if x[0] == "L"]
    assert len(ln) == len(lf) == 5000
    assert [x[1:3] + x[4:] for x in ln] == [x[1:3] + x[4:] for x in lf]  # source, orientations, overlap
    gap_near = [int(x[3]) - int(x[1]) for x in ln]
    gap_far = [abs(int(x[3]) - int(x[1])) for x in lf]
    assert all(0 <= g <= 64 for g in gap_near)
    assert sum(g > 64 for g in gap_far) > 4000
