"""The S-first hash dictionary on the lean front end (k_tile_lean kLeanClaim / kLeanEdges): inputs
whose S lines come first with unique names that are not the decimal ids.  The claim pass gives
node id = S index (builders.py:190-198: a key's first touch is its S line), the edge pass finds
both names of every edge line from the staged tile and writes the stream-order COO.  Every case
is compared with the oracle (and with the classic hash tiers, TEST_NO_HASH_LEAN); the cases that
break the premise — a repeated S name, an S line after an edge line, an edge key no S line
names, an unsupported record, a line outside the lean shapes — must fall back and still match.
"""
import random

import pytest

from test_gpu_diff import gpu_run, oracle_run, outcome

pytestmark = pytest.mark.gpu

MODES = [{}, {"directed": False}, {"asymmetric": True}]


def _names(r, n, width):
    out, seen = [], set()
    while len(out) < n:
        k = "".join(r.choice("abcdefghijklmnopqrstuvwxyz0123456789_") for _ in range(r.randint(*width)))
        if k not in seen:
            seen.add(k)
            out.append(k)
    return out


def _gfa(seed, n_s, n_l, width=(3, 12), ov="0M"):
    r = random.Random(seed)
    names = _names(r, n_s, width)
    lines = [f"S\t{k}\t{'ACGT' * r.randint(0, 3)}\n" for k in names]
    for _ in range(n_l):
        a = r.randrange(n_s)
        b = min(n_s - 1, a + r.randint(0, 5))
        lines.append(f"L\t{names[a]}\t{r.choice('+-')}\t{names[b]}\t{r.choice('+-')}\t{ov}\n")
    return names, lines


def _case(name):
    names, L = _gfa(11, 6000, 30000)
    if name == "canonical":
        return L, True
    if name == "p_and_header_lines":
        return ["H\tVN:Z:1.0\n"] + L[:6000] + ["P\tp1\t" + names[0] + "+," + names[1] + "-\t*\n"] + L[6000:], True
    if name == "names_of_16_and_17_bytes":  # inline head only / one tail byte compared in the input
        names, L = _gfa(12, 3000, 12000, width=(16, 17), ov="*")
        return L, True
    if name == "empty_name":
        return L[:10] + ["S\t\tACGT\n"] + L[10:6000] + ["L\t\t+\t" + names[3] + "\t-\t0M\n"] + L[6000:], True
    if name == "name_only_s_line":
        return L[:5] + ["S\tlonely\n"] + L[5:6000] + ["L\tlonely\t+\t" + names[3] + "\t-\t0M\n"] + L[6000:], True
    if name == "repeated_s_name":
        return L[:6000] + ["S\t" + names[77] + "\tAC\n"] + L[6000:], False
    if name == "s_after_edges":
        return L[:100] + L[6000:6100] + L[100:6000] + L[6100:], False
    if name == "edge_to_undefined_name":
        return L[:7000] + ["L\tnobody\t+\t" + names[3] + "\t-\t0M\n"] + L[7000:], False
    if name == "unsupported_record":
        return L[:7000] + ["W\tsample\t1\tchr1\t0\t10\t>x\n"] + L[7000:], False
    if name == "malformed_link":
        return L[:7000] + ["L\t" + names[1] + "\t+\n"] + L[7000:], False
    # the passes' tile lists (k_tile_lists): no edge line at all; tiles holding only P lines at the
    # end (claim list, no edge list); an S line in a tile far past the edge-only tiles
    if name == "s_lines_only":
        return L[:6000], True
    if name == "p_only_tiles_at_end":
        return L + ["P\tp%d\t%s+,%s-\t*\n" % (i, names[i], names[i + 1]) for i in range(4000)], True
    if name == "s_line_in_a_late_tile":
        return L[:6000] + L[6000:] + ["S\tlate_one\tAC\n"] + L[6000:9000], False
    raise KeyError(name)


CASES = ["canonical", "p_and_header_lines", "names_of_16_and_17_bytes", "empty_name", "name_only_s_line",
         "repeated_s_name", "s_after_edges", "edge_to_undefined_name", "unsupported_record", "malformed_link",
         "s_lines_only", "p_only_tiles_at_end", "s_line_in_a_late_tile"]


@pytest.mark.parametrize("case", CASES)
def test_hash_lean_equals_oracle(gpu, oracle_lib, monkeypatch, case):
    from gfa2network_amd import _native as nat

    lines, eligible = _case(case)
    data = "".join(lines).encode()
    for mode in MODES:
        raw = nat.build_from_buffer(data, nat.make_options(**mode))
        ph = raw.phase_ms
        took = "insert_lookup" in ph and "parse" not in ph
        if raw.status == 0:
            assert took == eligible, (case, mode, sorted(ph))
        for dtype in ("float64", "int8", "bool"):
            a = outcome(gpu_run(data, mode, dtype, None))
            assert a == outcome(oracle_run(oracle_lib, data, mode, dtype, None)), (case, mode, dtype)
            monkeypatch.setattr(nat, "TEST_FLAGS", nat.TEST_NO_HASH_LEAN)
            assert a == outcome(gpu_run(data, mode, dtype, None)), (case, mode, dtype, "classic")
            monkeypatch.setattr(nat, "TEST_FLAGS", 0)


def test_hash_lean_synthetic_large_equals_classic(gpu, monkeypatch):
    """10^7 edges of the synthetic generator with hashed names: the lean hash pass against the
    classic hash tiers, bit for bit, CSR and COO outputs."""
    from gfa2network_amd import _native as nat
    from gfa2network_amd import synth

    data = synth.host_bytes(2_000_000, 8_000_000, seed=5, names="hashed")
    for mode in ({}, {"directed": False}):
        raw = nat.build_from_buffer(data, nat.make_options(**mode))
        assert raw.status == 0 and "parse" not in raw.phase_ms, sorted(raw.phase_ms)
        a = outcome(gpu_run(data, mode, "float64", None))
        monkeypatch.setattr(nat, "TEST_FLAGS", nat.TEST_NO_HASH_LEAN)
        b = outcome(gpu_run(data, mode, "float64", None))
        monkeypatch.setattr(nat, "TEST_FLAGS", 0)
        assert a == b, mode
