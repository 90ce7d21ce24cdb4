"""Real-world GFA shapes on the tile-local lean parse (round 5): decimal-id files whose S lines carry
long sequences, whose P lines list thousands of steps, and that hold records the reference skips with
its one-shot warning (GFA 1.1 W lines, comments, blank lines; parser.py:114-131).  Such files took
the full parse (K1 + k_tile_parse) before: a line running past a tile's staged window, or any
unsupported record, failed the lean pass.  Now an S / P / O line needs only its first fields in view,
and the first unsupported record (ASCII first byte) is located per tile and ranked after the tile
scan (k_tile_lean_check).  Every case x mode x dtype equals the oracle and the full parse
(TEST_NO_TILE_LOCAL); the eligible ones must take the tile-local path ("tiles" phase absent).
"""
import random

import pytest

from test_gpu_diff import gpu_run, oracle_run, outcome

pytestmark = pytest.mark.gpu

MODES = [({}, None), ({"directed": False}, None), ({"asymmetric": True}, None), ({"bidirected": True}, None),
         ({"directed": False}, "RC"), ({"bidirected": True, "keep_directed_bidir": True}, "RC")]


def _seq(r, n):
    return "".join(r.choice("ACGT") for _ in range(n))


def _case(name):
    r = random.Random(sum(name.encode()))
    n_s = 4000
    S = []
    for k in range(1, n_s + 1):
        ln = r.choice([0, 3, 12, 40]) if r.random() < 0.97 else r.choice([2500, 9000, 40000])
        S.append(f"S\t{k}\t{_seq(r, ln) if ln else '*'}\tLN:i:{ln}\n")

    def link():
        a = r.randint(1, n_s)
        b = min(n_s, a + r.randint(0, 4))
        return f"L\t{a}\t{r.choice('+-')}\t{b}\t{r.choice('+-')}\t0M\tRC:i:{r.randint(1, 60)}\n"
    L = [link() for _ in range(16000)]
    P = ["P\tpath%d\t%s\t*\n" % (i, ",".join(f"{r.randint(1, n_s)}{r.choice('+-')}" for _ in range(r.choice([5, 9000]))))
         for i in range(6)]
    W = "W\tsample\t1\tchr1\t0\t100\t>1>2<3\n"
    if name == "long_sequences":
        return ["H\tVN:Z:1.0\n"] + S + L, True
    if name == "long_paths_between":
        return ["H\tVN:Z:1.0\n"] + S + P + L, True
    if name == "w_lines":
        return ["H\tVN:Z:1.1\n"] + S + L[:5000] + [W] * 3 + L[5000:] + [W], True
    if name == "comment_first":
        return ["# made by a tool\n"] + S + L, True
    if name == "blank_line":
        return S[:1000] + ["\n"] + S[1000:] + L, True
    if name == "w_in_many_tiles":
        return S + [W + x for x in L[::1000]] + L, True
    if name == "non_ascii_record":
        return S + L[:3000] + ["\xe9x\t1\n"] + L[3000:], False
    if name == "warn_then_malformed":
        return S + [W] + L[:3000] + ["L\t1\t+\n"] + L[3000:], False
    if name == "long_edge_line":  # an edge line past the window (a huge tag): the full parse
        return S + L[:3000] + ["L\t1\t+\t2\t-\t0M\tXX:Z:" + "q" * 50000 + "\n"] + L[3000:], False
    raise KeyError(name)


CASES = ["long_sequences", "long_paths_between", "w_lines", "comment_first", "blank_line", "w_in_many_tiles",
         "non_ascii_record", "warn_then_malformed", "long_edge_line"]


@pytest.mark.parametrize("case", CASES)
def test_lean_real_world_shapes_equal_oracle(gpu, oracle_lib, monkeypatch, case):
    from gfa2network_amd import _native as nat

    lines, eligible = _case(case)
    data = "".join(lines).encode("latin-1")
    for mode, wt in MODES:
        raw = nat.build_from_buffer(data, nat.make_options(weight_tag=wt, **mode))
        if raw.status == 0:
            took = "tiles" not in raw.phase_ms and "parse" in raw.phase_ms
            assert took == eligible, (case, mode, wt, sorted(raw.phase_ms))
        for dtype in ("float64", "int8", "bool"):
            a = outcome(gpu_run(data, mode, dtype, wt))
            assert a == outcome(oracle_run(oracle_lib, data, mode, dtype, wt)), (case, mode, wt, dtype)
            monkeypatch.setattr(nat, "TEST_FLAGS", nat.TEST_NO_TILE_LOCAL)
            assert a == outcome(gpu_run(data, mode, dtype, wt)), (case, mode, wt, dtype, "full parse")
            monkeypatch.setattr(nat, "TEST_FLAGS", 0)
