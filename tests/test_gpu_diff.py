"""GPU vs the oracle on inputs the reference's own fixtures do not cover.

* randomized GFA texts full of parse quirks (fuzz_gfa.make), every mode x dtype family;
* the synthetic generator at 10^5 - 10^7 edges, bit-exact COO / CSR / MAX-SYM / names;
* bench-size properties (C4: 200M edges) that hold whatever the size: symmetry of the
  MAX-SYM CSR, canonical CSR, node names = "1".."N" in S order.
"""
import io

import numpy as np
import pytest
import scipy.sparse as sp

import fuzz_gfa
import golden_util as G

pytestmark = pytest.mark.gpu

MODES = [
    {},
    {"directed": False},
    {"asymmetric": True},
    {"bidirected": True},
    {"bidirected": True, "keep_directed_bidir": True},
    {"keep_directed_bidir": True, "asymmetric": True},
    {"strip_orientation": True, "bidirected": True},
]


def outcome(run):
    res, exc, warns, so, se = G.run_python(run)
    if exc is not None:
        return ("exc", type(exc).__name__, str(exc), tuple(w["msg"] for w in warns), so, se)
    A, nodes = res
    M = A.tocoo() if A.format == "csr" else A
    key = [A.format, str(A.dtype), A.shape, tuple(w["msg"] for w in warns), so, se, nodes]
    if A.format == "coo":
        key += [A.row.tobytes(), A.col.tobytes(), A.data.tobytes()]
    else:
        key += [A.indptr.tobytes(), A.indices.tobytes(), A.data.tobytes()]
    del M
    return tuple(key)


def gpu_run(data: bytes, mode: dict, dtype: str, wt, raw_bytes_id=True, verbose=False):
    import io

    from gfa2network_amd import parse_gfa

    return lambda: parse_gfa(io.BytesIO(data), build_graph=False, build_matrix=True, return_node_list=True,
                             raw_bytes_id=raw_bytes_id, verbose=verbose, dtype=dtype, weight_tag=wt, **mode)


def oracle_run(oracle_mod, data: bytes, mode: dict, dtype: str, wt, raw_bytes_id=True, verbose=False):
    from gfa2network_amd.api import finalize

    def run():
        o = oracle_mod.run(data, dtype=dtype, weight_tag=wt, **mode)
        return finalize(oracle_mod.to_raw(o, "parse"), dtype=np.dtype(dtype), return_node_list=True,
                        raw_bytes_id=raw_bytes_id, verbose=verbose)

    return run


@pytest.mark.parametrize("block", range(8))
def test_fuzz_gpu_equals_oracle(gpu, oracle_lib, block):
    bad = []
    for seed in range(block * 40, block * 40 + 40):
        data = fuzz_gfa.make(seed, n_lines=50, allow_errors=seed % 3 == 0)
        mode = MODES[seed % len(MODES)]
        dtype = ["float64", "float32", "int8", "int32", "bool"][seed % 5]
        for wt in (None, "RC"):
            for rbi in (True, False):
                a = outcome(gpu_run(data, mode, dtype, wt, rbi, verbose=seed % 2 == 0))
                b = outcome(oracle_run(oracle_lib, data, mode, dtype, wt, rbi, verbose=seed % 2 == 0))
                if a != b:
                    bad.append((seed, mode, dtype, wt, rbi, a[:3], b[:3]))
    assert not bad, bad[:3]


def test_fuzz_convert_format_equals_oracle(gpu, oracle_lib):
    """convert_format(A, "csr") on the GPU == scipy's tocsr, on the COO outputs."""
    from gfa2network_amd import convert_format

    bad = []
    for seed in range(300, 420):
        data = fuzz_gfa.make(seed, n_lines=80, allow_errors=False)
        for dtype in ("float64", "float32", "int8", "bool"):
            o = oracle_lib.run(data, dtype=dtype, weight_tag="RC", directed=False)
            if o.status:
                continue
            A = sp.coo_matrix((o.data, (o.rows.astype(np.int32), o.cols.astype(np.int32))),
                              shape=(o.n_nodes, o.n_nodes), dtype=dtype)
            C = convert_format(A, "csr")
            R = A.tocsr()
            if not (C.indptr.tobytes() == R.indptr.tobytes() and C.indices.tobytes() == R.indices.tobytes()
                    and C.data.tobytes() == R.data.tobytes() and C.dtype == R.dtype):
                bad.append((seed, dtype))
            Cc = convert_format(A, "csc")
            Rc = A.tocsc()
            if not (Cc.indptr.tobytes() == Rc.indptr.tobytes() and Cc.indices.tobytes() == Rc.indices.tobytes()
                    and Cc.data.tobytes() == Rc.data.tobytes()):
                bad.append((seed, dtype, "csc"))
    assert not bad, bad[:5]


@pytest.mark.parametrize("n_s,n_l,rc,far", [(1000, 4000, True, False), (100_000, 400_000, True, False),
                                             (1_000_000, 4_000_000, False, False), (100_000, 400_000, False, True),
                                             (1_000_000, 4_000_000, False, True)])
def test_synthetic_gpu_equals_oracle(gpu, oracle_lib, n_s, n_l, rc, far):
    """far: L lines' second segment uniform over all segments — no entry's two rows share a finish
    bucket, so the partition carries no pair elements (g2n_sym.hip); otherwise nearly all do."""
    from gfa2network_amd import synth

    data = synth.host_bytes(n_s, n_l, seed=11, rc_tag=rc, far_links=far)
    modes = MODES if n_l <= 400_000 else [{}, {"directed": False}, {"bidirected": True}]
    for mode in modes:
        for dtype in (["float64", "float32", "int32", "int8"] if n_l <= 400_000 else ["float64"]):
            wt = "RC" if rc else None
            a = outcome(gpu_run(data, mode, dtype, wt))
            b = outcome(oracle_run(oracle_lib, data, mode, dtype, wt))
            assert a == b, (mode, dtype)


def test_float_duplicate_sums_match_scipy_order(gpu, oracle_lib):
    """Rows of > 16 entries with >= 3 inexact float duplicates: the GPU re-runs scipy's
    std::sort order (stl_sort.h) and matches scipy bit for bit."""
    import random

    r = random.Random(5)
    lines = []
    vals = ["1e16", "1", "-1e16", "0.1", "3.3", "-2.7", "1e-3", "7.25", "1e300", "-1e300"]
    for _ in range(4000):
        lines.append(f"L\tr{r.randint(0, 6)}\t+\tc{r.randint(0, 40)}\t+\t*\tRC:f:{r.choice(vals)}\n")
    data = "".join(lines).encode()
    for mode in ({}, {"directed": False}, {"asymmetric": True}):
        for dtype in ("float64", "float32"):
            a = outcome(gpu_run(data, mode, dtype, "RC"))
            b = outcome(oracle_run(oracle_lib, data, mode, dtype, "RC"))
            assert a == b, (mode, dtype)
    from gfa2network_amd import convert_format, parse_gfa
    import io

    A = parse_gfa(io.BytesIO(data), build_graph=False, build_matrix=True, directed=False, weight_tag="RC")
    C, R = convert_format(A, "csr"), A.tocsr()
    assert C.data.tobytes() == R.data.tobytes() and C.indices.tobytes() == R.indices.tobytes()


def test_c4_properties_on_device(gpu):
    """Full C4 size (50M S / 200M L, 6.3 GB) on the device: size-independent properties."""
    import ctypes

    from gfa2network_amd import _native as nat
    from gfa2network_amd import synth

    lib = nat.load()
    dev = synth.DeviceInput(50_000_000, 200_000_000, seed=0)
    ctx = lib.g2n_context_create(0)
    try:
        opts = nat.make_options(output=nat.OUT_CSR)
        res = nat.Result()
        assert lib.g2n_build_device(ctx, dev.ptr, dev.len, ctypes.byref(opts), ctypes.byref(res)) == 0
        n, nnz = res.n_nodes, res.nnz
        assert res.n_edges == 200_000_000 and n == 50_000_000 and res.format == nat.FMT_CSR
        indptr = np.empty(n + 1, np.int32)
        indices = np.empty(nnz, np.int32)
        hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime libg2n.so loaded (its SONAME)
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        assert hip.hipMemcpy(indptr.ctypes.data, res.indptr, indptr.nbytes, 2) == 0
        assert hip.hipMemcpy(indices.ctypes.data, res.indices, indices.nbytes, 2) == 0
        offs = np.empty(n + 1, np.int64)
        assert hip.hipMemcpy(offs.ctypes.data, res.names_offsets, offs.nbytes, 2) == 0
        blob = np.empty(int(offs[-1]), np.uint8)
        assert hip.hipMemcpy(blob.ctypes.data, res.names_blob, blob.nbytes, 2) == 0
    finally:
        lib.g2n_context_destroy(ctx)
        dev.free()
    assert indptr[0] == 0 and indptr[-1] == nnz and np.all(np.diff(indptr) >= 0)
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(indptr))
    k1 = rows * n + indices  # canonical CSR: strictly increasing (row, col)
    assert np.all(np.diff(k1) > 0)
    k2 = np.sort(indices.astype(np.int64) * n + rows)
    assert np.array_equal(k1, k2)  # MAX-SYM result is structurally symmetric
    # S lines define "1".."N" in order, so node k is named str(k+1)
    names = blob.tobytes()
    want = "".join(str(k) for k in range(1, n + 1)).encode()
    assert names == want


def _canonical_gfa(seed: int, n_s: int, n_l: int, long_names: bool, interleave: bool = False) -> bytes:
    """S lines first (distinct names, some longer than the 16 inline key bytes), then L lines
    that only name defined segments: the input the S-first dictionary fast path is for.
    interleave: S and L lines mixed, every L line naming segments defined above it."""
    import random

    r = random.Random(seed)
    names = []
    for k in range(n_s):
        if long_names and k % 3 == 0:
            names.append(f"chr{r.randint(1, 22)}_segment_{k:08d}_" + "x" * r.randint(0, 40))
        else:
            names.append(f"{k + 1}")

    def link(pool):
        a, b = r.choice(pool), r.choice(pool)
        return f"L\t{a}\t{r.choice('+-')}\t{b}\t{r.choice('+-')}\t*\tRC:i:{r.randint(-3, 9)}\n"

    lines = [f"H\tVN:Z:1.0\n"]
    if interleave:
        per = max(1, n_l // n_s)
        for k, n in enumerate(names):
            lines.append(f"S\t{n}\t*\n")
            lines += [link(names[:k + 1]) for _ in range(per)]
    else:
        lines += [f"S\t{n}\t*\n" for n in names]
        lines += [link(names) for _ in range(n_l)]
    return "".join(lines).encode()


def _phases(data: bytes, **kw):
    from gfa2network_amd import _native as nat

    raw = nat.build_from_buffer(data, nat.make_options(**kw))
    return raw.status, raw.phase_ms


@pytest.mark.parametrize("long_names,interleave", [(False, False), (True, False), (True, True)])
def test_s_first_fast_path_taken_and_exact(gpu, oracle_lib, long_names, interleave):
    data = _canonical_gfa(7 + long_names, 3000, 12000, long_names, interleave)
    for mode in MODES:
        st, ph = _phases(data, **mode)
        # decimal names: the lean parse needs no dictionary phase at all; long names: the S-first table
        assert st == 0 and "ids_general" not in ph and ("ids_fast" in ph or not long_names), (mode, sorted(ph))
        for dtype, wt in (("float64", "RC"), ("int8", None), ("float32", "RC")):
            a = outcome(gpu_run(data, mode, dtype, wt))
            b = outcome(oracle_run(oracle_lib, data, mode, dtype, wt))
            assert a == b, (mode, dtype, wt)


@pytest.mark.parametrize("case", ["l_before_s", "missing_segment", "duplicate_s"])
def test_s_first_fallback_to_general_dictionary(gpu, oracle_lib, case):
    """Inputs where a key's first touch is not its S line: the fast path must notice and the
    general insert rounds must give the reference's first-touch ids."""
    base = _canonical_gfa(3, 500, 3000, True).decode().splitlines(keepends=True)
    s_lines = [x for x in base if x.startswith("S")]
    l_lines = [x for x in base if x.startswith("L")]
    if case == "l_before_s":
        text = l_lines[:50] + s_lines + l_lines[50:]
    elif case == "missing_segment":
        text = s_lines + l_lines[:100] + ["L\tnot_a_segment\t+\t1\t-\t*\tRC:i:2\n"] + l_lines[100:]
    else:  # a later S line repeats an earlier name
        text = s_lines + [s_lines[10], s_lines[0]] + l_lines
    data = "".join(text).encode()
    for mode in MODES:
        st, ph = _phases(data, **mode)
        assert st == 0
        if case != "duplicate_s":  # there the earlier S line may win the claim: fast path stays exact
            assert "ids_general" in ph, (case, mode, sorted(ph))
        for dtype, wt in (("float64", "RC"), ("int32", None)):
            a = outcome(gpu_run(data, mode, dtype, wt))
            b = outcome(oracle_run(oracle_lib, data, mode, dtype, wt))
            assert a == b, (case, mode, dtype, wt)


def test_general_dictionary_forced(gpu, oracle_lib, monkeypatch):
    """TEST_DICT_GENERAL keeps the general insert rounds covered on canonical inputs too."""
    from gfa2network_amd import _native as nat

    monkeypatch.setattr(nat, "TEST_FLAGS", nat.TEST_DICT_GENERAL)
    data = _canonical_gfa(11, 2000, 8000, True)
    for mode in MODES:
        st, ph = _phases(data, **mode)
        assert st == 0 and "ids_general" in ph and "ids_fast" not in ph
        a = outcome(gpu_run(data, mode, "float64", "RC"))
        b = outcome(oracle_run(oracle_lib, data, mode, "float64", "RC"))
        assert a == b, mode


def test_long_runs_of_empty_rows(gpu, oracle_lib):
    """Thousands of consecutive node ids with no entries in a row (or column): the row-start
    pass falls back to a binary search per row; the CSR must not change."""
    import io
    import random

    from gfa2network_amd import convert_format, parse_gfa

    r = random.Random(2)
    lines = [f"S\t{k}\t*\n" for k in range(1, 3001)]
    lines += [f"L\t{r.randint(1, 10)}\t+\t{r.randint(2990, 3000)}\t-\t*\tRC:i:{r.randint(1, 5)}\n"
              for _ in range(500)]
    data = "".join(lines).encode()
    for mode in ({}, {"directed": False}, {"bidirected": True}):
        a = outcome(gpu_run(data, mode, "float64", "RC"))
        b = outcome(oracle_run(oracle_lib, data, mode, "float64", "RC"))
        assert a == b, mode
    A = parse_gfa(io.BytesIO(data), build_graph=False, build_matrix=True, directed=False, weight_tag="RC")
    for fmt, ref in (("csr", A.tocsr()), ("csc", A.tocsc())):
        C = convert_format(A, fmt)
        assert C.indptr.tobytes() == ref.indptr.tobytes() and C.indices.tobytes() == ref.indices.tobytes()
        assert C.data.tobytes() == ref.data.tobytes()


def test_field_boundaries_near_mask_span_and_tiles(gpu, oracle_lib):
    """Lines of 40-90 bytes (the field masks cover 64), names ending near byte 64, and S lines
    long enough to cross a 32 KiB tile and its halo: the LDS front end must match the oracle."""
    import random

    r = random.Random(9)
    names = []
    lines = []
    for k in range(400):
        n = f"n{k}_" + "a" * r.randint(0, 70)
        names.append(n)
        seq = "ACGT" * r.choice([0, 1, 10, 3000, 9000])  # up to 36 KB: crosses tiles and halos
        lines.append(f"S\t{n}\t{seq or '*'}\tLN:i:{len(seq)}\n")
    for _ in range(3000):
        a, b = r.choice(names), r.choice(names)
        tags = "\t".join(f"X{q}:i:{r.randint(0, 9)}" for q in range(r.randint(0, 4)))
        w = f"\tRC:i:{r.randint(-5, 50)}" if r.random() < 0.8 else ""
        lines.append(f"L\t{a}\t{r.choice('+-')}\t{b}\t{r.choice('+-')}\t{r.randint(0, 99)}M{w}" +
                     (f"\t{tags}" if tags else "") + "\n")
    r.shuffle(lines)  # S lines after the links that name them: the general dictionary too
    data = "".join(lines).encode()
    for mode in MODES[:4]:
        for wt in (None, "RC"):
            a = outcome(gpu_run(data, mode, "float64", wt))
            b = outcome(oracle_run(oracle_lib, data, mode, "float64", wt))
            assert a == b, (mode, wt)


def _decimal_gfa(seed: int, n_s: int, n_l: int) -> list[str]:
    import random

    r = random.Random(seed)
    lines = ["H\tVN:Z:1.0\n"] + [f"S\t{k}\t{'ACGT'[k % 4] * (k % 5)}\n" for k in range(1, n_s + 1)]
    lines += [f"L\t{r.randint(1, n_s)}\t{r.choice('+-')}\t{r.randint(1, n_s)}\t{r.choice('+-')}\t0M"
              f"\tRC:i:{r.randint(1, 9)}\n" for _ in range(n_l)]
    return lines


DECIMAL_CASES = {
    "canonical": lambda L: L,
    "s_leading_zero": lambda L: L[:5] + ["S\t05\t*\n"] + L[6:],  # line 5 named "05", not "5"
    "s_out_of_order": lambda L: L[:3] + [L[4], L[3]] + L[5:],
    "s_after_l": lambda L: [x for x in L if not x.startswith("S\t9")] + [x for x in L if x.startswith("S\t9")],
    "s_duplicate": lambda L: L + ["S\t1\t*\n"],
    "edge_new_node": lambda L: L[:700] + ["L\t99999\t+\t1\t-\t0M\n"] + L[700:],
    "edge_leading_zero": lambda L: L[:700] + ["L\t007\t+\t1\t-\t0M\n"] + L[700:],
    "edge_zero": lambda L: L[:700] + ["L\t0\t+\t1\t-\t0M\n"] + L[700:],
    "edge_eleven_digits": lambda L: L[:700] + ["L\t12345678901\t+\t1\t-\t0M\n"] + L[700:],
    "edge_odd_orientation": lambda L: L[:700] + ["L\t3\t*\t4\t-\t0M\n"] + L[700:],
    "edge_plus_sign": lambda L: L[:700] + ["L\t+3\t+\t4\t-\t0M\n"] + L[700:],
    "edge_embedded_orientation": lambda L: L[:700] + ["L\t3+\t4-\t0M\t*\n"] + L[700:],
    "s_name_hex": lambda L: L[:2] + ["S\t0x2\t*\n"] + L[3:],
}


@pytest.mark.parametrize("case", sorted(DECIMAL_CASES))
def test_decimal_id_dictionary(gpu, oracle_lib, case):
    """S lines naming "1".."N" in order give ids by arithmetic in the parse; every input that breaks
    the premise falls back to the hash dictionary.  Either way the result is the oracle's."""
    data = "".join(DECIMAL_CASES[case](_decimal_gfa(4, 400, 2400))).encode()
    for mode in MODES:
        st, ph = _phases(data, **mode)
        assert st == 0
        took = "table_init" not in ph and "ids_general" not in ph
        if case == "canonical":
            assert took, (mode, sorted(ph))
        elif case not in ("edge_odd_orientation", "edge_embedded_orientation"):
            assert not took, (case, mode, sorted(ph))
        for dtype, wt in (("float64", "RC"), ("int32", None)):
            a = outcome(gpu_run(data, mode, dtype, wt))
            b = outcome(oracle_run(oracle_lib, data, mode, dtype, wt))
            assert a == b, (case, mode, dtype, wt)


TILE_LOCAL_CASES = {  # inputs of ~60 tiles: the premise checked ACROSS tiles after the tile-local parse
    "canonical": lambda L: L,
    "s_renamed_late": lambda L: L[:15001] + ["S\t15001x\t*\n"] + L[15002:],  # a later tile's S name
    "s_skips_a_number": lambda L: L[:9000] + L[9001:],  # S lines 1..8999, 9001..: ids off by one
    "edge_between_s_tiles": lambda L: L[:12000] + [L[-1]] + L[12000:],  # an L line before later S lines
    "edge_names_n_plus_1": lambda L: L + ["L\t20001\t+\t1\t-\t0M\n"],  # no such S line (N = 20000)
    "long_line_deferred": lambda L: L[:30000] + ["L\t1\t+\t2\t-\t0M\tXX:Z:" + "a" * 40000 + "\n"] + L[30000:],
}


@pytest.mark.parametrize("case", sorted(TILE_LOCAL_CASES))
def test_tile_local_parse_premise_across_tiles(gpu, oracle_lib, monkeypatch, case):
    """The decimal-id parse without K1 (tile-local positions; the premise checked per tile after one
    scan, then the COO compacted — or, for a CSR output of an unweighted build, left in group slots
    for the bucket partition) against the oracle, against the lean parse after K1
    (TEST_NO_TILE_LOCAL) and against per-tile slots (TEST_NO_GROUP); cases that break the premise
    only across tiles must fall back."""
    from gfa2network_amd import _native as nat

    data = "".join(TILE_LOCAL_CASES[case](_decimal_gfa(9, 20000, 80000))).encode()
    assert len(data) > 40 * 32768
    for mode in MODES:
        st, ph = _phases(data, **mode)
        assert st == 0
        local = "parse" in ph and "tiles" not in ph
        eligible = not mode.get("strip_orientation")  # (bidirected: the extended instance, round 5)
        assert local == (eligible and case == "canonical"), (case, mode, sorted(ph))
        for dtype, wt in (("float64", None), ("int8", None), ("float64", "RC")):
            a = outcome(gpu_run(data, mode, dtype, wt))
            assert a == outcome(oracle_run(oracle_lib, data, mode, dtype, wt)), (case, mode, dtype, wt)
            for flag in (nat.TEST_NO_TILE_LOCAL, nat.TEST_NO_GROUP):
                monkeypatch.setattr(nat, "TEST_FLAGS", flag)
                assert a == outcome(gpu_run(data, mode, dtype, wt)), (case, mode, dtype, wt, flag)
                monkeypatch.setattr(nat, "TEST_FLAGS", 0)


def test_decimal_ids_equal_hash_dictionary(gpu, monkeypatch):
    """The lean decimal-id parse (coordinates written by the parse), the non-lean one (TEST_NO_LEAN:
    ids per touch, then k_triplets) and the hash dictionary (TEST_DICT_HASH) agree bit for bit at
    10^7 edges, weighted and not, COO and CSR outputs."""
    from gfa2network_amd import _native as nat
    from gfa2network_amd import synth

    data = synth.host_bytes(2_000_000, 8_000_000, seed=3, rc_tag=True)
    for mode in ({}, {"directed": False}, {"bidirected": True}, {"bidirected": True, "keep_directed_bidir": True}):
        for wt in ("RC", None):
            st, ph = _phases(data, **mode)
            assert "values" in ph and "triplets" not in ph and "table_init" not in ph, sorted(ph)
            a = outcome(gpu_run(data, mode, "float64", wt))
            for flag in (nat.TEST_NO_LEAN, nat.TEST_DICT_HASH, nat.TEST_DICT_HASH | nat.TEST_NO_HASH_LEAN):
                monkeypatch.setattr(nat, "TEST_FLAGS", flag)
                st, ph = _phases(data, **mode)
                hashed = bool(flag & nat.TEST_DICT_HASH)
                # the lean S-first hash pass writes the COO itself (no triplets phase): plain builds and,
                # since round 5, bidirected ones (the extended edge pass)
                lean_hash = hashed and not (flag & nat.TEST_NO_HASH_LEAN)
                assert ("insert_lookup" in ph) == hashed and ("triplets" in ph) == (not lean_hash), \
                    (flag, mode, sorted(ph))
                b = outcome(gpu_run(data, mode, "float64", wt))
                monkeypatch.setattr(nat, "TEST_FLAGS", 0)
                assert a == b, (mode, wt, flag)


def test_maxsym_buckets_match_oracle_and_classic(gpu, oracle_lib, monkeypatch):
    """The fused bucket A.maximum(A.T) (k_maxsym_bucket) equals the oracle and the classic
    row-sum + merge path: hubs that overflow a bucket (classic fallback), heavy duplicate runs
    (int8 wrap-around to 0 and -128, bool), self loops, every CLI dtype."""
    import random

    from gfa2network_amd import _native as nat

    r = random.Random(12)
    lines = [f"S\t{k}\t*\n" for k in range(1, 6001)]
    lines += [f"L\t{r.randint(1, 6000)}\t+\t{r.randint(1, 6000)}\t-\t0M\n" for _ in range(30000)]
    lines += ["L\t7\t+\t9\t+\t0M\n"] * 256 + ["L\t9\t+\t7\t+\t0M\n"] * 128 + ["L\t11\t+\t11\t+\t0M\n"] * 300
    hub = [f"L\t5000\t+\t{k}\t+\t0M\n" for k in range(1, 6001)]  # > one bucket's capacity
    for extra in ([], hub):  # the hub: the group-slot COO is refused, the build redone without it
        data = "".join(lines + extra).encode()
        for mode in ({}, {"directed": False}):
            for dtype in ("bool", "int8", "int32", "float32", "float64"):
                a = outcome(gpu_run(data, mode, dtype, None))
                b = outcome(oracle_run(oracle_lib, data, mode, dtype, None))
                assert a == b, (dtype, bool(extra), mode)
                for flag in (nat.TEST_NO_BUCKETS, nat.TEST_NO_GROUP):
                    monkeypatch.setattr(nat, "TEST_FLAGS", flag)
                    c = outcome(gpu_run(data, mode, dtype, None))
                    monkeypatch.setattr(nat, "TEST_FLAGS", 0)
                    assert a == c, (dtype, bool(extra), mode, flag)


def test_maxsym_buckets_large(gpu, monkeypatch):
    """Bucket path == classic path at 10^7 edges (two partition passes), float64 and int8."""
    from gfa2network_amd import _native as nat
    from gfa2network_amd import synth

    data = synth.host_bytes(2_000_000, 8_000_000, seed=21)
    a = {dt: outcome(gpu_run(data, {}, dt, None)) for dt in ("float64", "int8")}
    monkeypatch.setattr(nat, "TEST_FLAGS", nat.TEST_NO_BUCKETS)
    b = {dt: outcome(gpu_run(data, {}, dt, None)) for dt in ("float64", "int8")}
    monkeypatch.setattr(nat, "TEST_FLAGS", 0)
    assert a == b


def test_builds_are_deterministic(gpu):
    """Atomics decide table slots, scatter positions and bucket cursors: two builds of the same
    input still give identical bytes, on every dictionary tier."""
    from gfa2network_amd import synth

    data = synth.host_bytes(300_000, 1_200_000, seed=4, rc_tag=True)
    hashed = data.replace(b"S\t1\t", b"S\tx1\t", 1)  # first S not "1": the hash tiers
    for d in (data, hashed):
        for mode, wt in (({}, None), ({"directed": False}, "RC"), ({"bidirected": True}, "RC")):
            assert outcome(gpu_run(d, mode, "float64", wt)) == outcome(gpu_run(d, mode, "float64", wt))


def _csr_cases():
    import random

    from gfa2network_amd import synth

    r = random.Random(3)
    dup = [f"S\t{k}\t*\n" for k in range(1, 3001)]
    dup += [f"L\t{r.randint(1, 3000)}\t+\t{r.randint(1, 3000)}\t-\t0M\tRC:i:{r.randint(-2, 3)}\n" for _ in range(20000)]
    dup += ["L\t7\t+\t9\t+\t0M\n"] * 256 + ["L\t9\t+\t7\t+\t0M\n"] * 128 + ["L\t11\t+\t11\t+\t0M\n"] * 300
    dup += [f"L\t2000\t+\t{k}\t+\t0M\n" for k in range(1, 3001)]  # a hub longer than a finish bucket
    return {"dups": "".join(dup).encode(), "synth": synth.host_bytes(200_000, 800_000, seed=7, rc_tag=True)}


@pytest.mark.parametrize("case", ["dups", "synth"])
def test_csr_output_equals_oracle(gpu, oracle_lib, case):
    """output = G2N_OUT_CSR (what convert_format(parse_gfa(...), "csr") returns, cli.py:239) in every
    mode and dtype family: unweighted SUM CSRs through the bucket partition (g2n_sym.hip, sum mode:
    int8 runs of 256 copies stay as explicit zeros), weighted ones through the row sums."""
    from gfa2network_amd import _native as nat

    data = _csr_cases()[case]
    bad = []
    for mode in MODES:
        for dtype in ("float64", "int8", "bool"):
            for wt in (None, "RC"):
                raw = nat.build_from_buffer(data, nat.make_options(output=nat.OUT_CSR, dtype=dtype, weight_tag=wt,
                                                                   **mode))
                o = oracle_lib.run(data, dtype=dtype, weight_tag=wt, **mode)
                if raw.status != o.status:
                    bad.append((mode, dtype, wt, raw.status, o.status))
                    continue
                if o.status:
                    continue
                R = oracle_lib.to_raw(o, "csr")
                if not (raw.indptr.tobytes() == R.indptr.tobytes() and raw.indices.tobytes() == R.indices.tobytes()
                        and raw.data.tobytes() == R.data.tobytes()):
                    bad.append((mode, dtype, wt))
    assert not bad, bad[:4]


def _weighted_sum_cases():
    import random

    r = random.Random(17)
    base = [f"S\t{k}\t*\n" for k in range(1, 4001)]
    ints = [f"L\t{r.randint(1, 4000)}\t+\t{r.randint(1, 4000)}\t-\t0M\tRC:i:{r.randint(-3, 5)}\n"
            for _ in range(24000)]
    ints += ["L\t7\t+\t9\t+\t0M\tRC:i:1\n"] * 300 + ["L\t9\t+\t7\t+\t0M\tRC:i:2\n"] * 130  # int8 wrap
    ints += ["L\t11\t+\t11\t+\t0M\tRC:i:-1\n", "L\t11\t+\t11\t+\t0M\tRC:i:1\n"] * 40  # sums to 0
    ints += ["L\t12\t+\t13\t+\t0M\n"] * 3  # no tag: weight 1
    hub = [f"L\t3000\t+\t{k}\t+\t0M\tRC:i:{k % 7}\n" for k in range(1, 4001)]  # > one bucket
    big = ["L\t20\t+\t21\t+\t0M\tRC:i:16777216\n"] * 2  # float32: a run past 2^24
    frac = ["L\t30\t+\t31\t+\t0M\tRC:f:0.5\n"]
    negz = ["L\t40\t+\t41\t+\t0M\tRC:f:-0.0\n"]
    # the dtypes whose SUM CSR must take the row sums (the cast of 0.5 / -0.0 to an integer dtype or bool
    # is an exact integer: those stay on the buckets)
    every, floats = {"float64", "float32", "int32", "int8", "bool"}, {"float64", "float32"}
    return {"ints": (base + ints, set()), "hub": (base + ints + hub, every), "big": (base + ints + big, {"float32"}),
            "frac": (base + ints + frac, floats), "negzero": (base + ints + negz, floats)}


@pytest.mark.parametrize("case", ["ints", "hub", "big", "frac", "negzero"])
def test_weighted_sum_buckets_match_oracle_and_classic(gpu, oracle_lib, monkeypatch, case):
    """Weighted SUM CSRs (coo.tocsr, utils.py:55) through the value-carrying bucket partition (passes
    5 / 6, k_sumw_finish): integer weights in every dtype family equal the oracle and the stable row-sum
    path (TEST_NO_BUCKETS) byte for byte; a premise break — a fractional or -0.0 value, a float32 run
    whose magnitudes pass 2^24, a bucket past its capacity — takes the row sums (sum_buckets False)."""
    from gfa2network_amd import _native as nat

    lines, rowsum = _weighted_sum_cases()[case]
    data = "".join(lines).encode()
    bad = []
    for mode in ({}, {"directed": False}, {"bidirected": True}, {"asymmetric": True}):
        for dtype in ("float64", "float32", "int32", "int8", "bool"):
            o = oracle_lib.run(data, dtype=dtype, weight_tag="RC", **mode)
            raw = nat.build_from_buffer(data, nat.make_options(output=nat.OUT_CSR, dtype=dtype, weight_tag="RC",
                                                               **mode))
            if raw.status != o.status:
                bad.append((mode, dtype, "status", raw.status, o.status))
                continue
            if o.status or raw.format != "csr":
                continue
            R = oracle_lib.to_raw(o, "csr")
            same = (np.array_equal(raw.indptr, R.indptr) and np.array_equal(raw.indices, R.indices)
                    and raw.data.tobytes() == R.data.tobytes())
            if not same:
                bad.append((mode, dtype, "oracle"))
            want = dtype not in rowsum and mode != {}  # {}: MAX-SYM (weighted: the row sums)
            if raw.sum_buckets != want:
                bad.append((mode, dtype, "path", raw.sum_buckets))
            monkeypatch.setattr(nat, "TEST_FLAGS", nat.TEST_NO_BUCKETS)
            c = nat.build_from_buffer(data, nat.make_options(output=nat.OUT_CSR, dtype=dtype, weight_tag="RC",
                                                             **mode))
            monkeypatch.setattr(nat, "TEST_FLAGS", 0)
            if c.sum_buckets or not (np.array_equal(raw.indptr, c.indptr) and np.array_equal(raw.indices, c.indices)
                                     and raw.data.tobytes() == c.data.tobytes()):
                bad.append((mode, dtype, "classic"))
    assert not bad, bad[:4]


@pytest.mark.parametrize("mode", [{}, {"directed": False}, {"bidirected": True}])
def test_failed_build_leaves_no_call_state(gpu, oracle_lib, mode):
    """A build that throws after its parse and ids (TEST_THROW_AFTER_IDS: the group-slot COO active, the
    names launch deferred to the side stream) must leave nothing behind on the device's shared context:
    the next convert_format and the next build on it equal the oracle."""
    from gfa2network_amd import _native as nat
    from gfa2network_amd import synth

    data = synth.host_bytes(20_000, 80_000, seed=5)
    with pytest.raises(RuntimeError, match="injected"):
        nat.build_from_buffer(data, nat.make_options(output=nat.OUT_CSR, want_node_names=True,
                                                     test_flags=nat.TEST_THROW_AFTER_IDS, **mode))
    o = oracle_lib.run(data, **mode)
    R = oracle_lib.to_raw(o, "csr")  # what convert_format(parse_gfa(...), "csr") returns
    n = int(o.n_nodes)
    C = sp.coo_matrix((o.data, (o.rows.astype(np.int32), o.cols.astype(np.int32))), shape=(n, n)).tocsr()
    got = nat.coo_to_csr(o.rows, o.cols, o.data, n, n)  # convert_format of the stream-order COO
    ok = np.array_equal(got.indptr, C.indptr) and np.array_equal(got.indices, C.indices)
    ok = ok and got.data.tobytes() == C.data.tobytes()
    assert ok
    with pytest.raises(RuntimeError, match="injected"):
        nat.build_from_buffer(data, nat.make_options(output=nat.OUT_CSR, want_node_names=True,
                                                     test_flags=nat.TEST_THROW_AFTER_IDS, **mode))
    raw = nat.build_from_buffer(data, nat.make_options(output=nat.OUT_CSR, want_node_names=True, **mode))
    assert raw.status == 0
    ok = np.array_equal(raw.indptr, R.indptr) and np.array_equal(raw.indices, R.indices)
    ok = ok and raw.data.tobytes() == R.data.tobytes()
    assert ok
    assert np.array_equal(raw.names_blob, o.names_blob)


@pytest.mark.parametrize("case", ["synth_dense", "synth"])
def test_int64_index_path_equals_oracle(gpu, oracle_lib, case):
    """TEST_INDEX64 forces the CSR results of unweighted builds through the int64 index path (what a
    result of more than 2^31 - 1 entries takes: scipy's get_index_dtype, utils.py:55, builders.py:283):
    int64 indptr / indices holding exactly the oracle's values, in every mode (MAX-SYM, SUM twins,
    bidirected) and dtype family."""
    from gfa2network_amd import _native as nat

    # (inputs the bucket partition takes: a bucket past its LDS capacity — the "dups" hubs — goes the
    # int32 row-sum path, whose results stay below 2^31 entries; synth_dense: ~20 copies per pair)
    from gfa2network_amd import synth

    data = synth.host_bytes(3000, 60000, seed=9) if case == "synth_dense" else _csr_cases()[case]
    bad = []
    for mode in MODES:
        for dtype in ("float64", "int8", "bool"):
            for out in (nat.OUT_CSR, nat.OUT_PARSE):
                o = oracle_lib.run(data, dtype=dtype, **mode)
                raw = nat.build_from_buffer(data, nat.make_options(output=out, dtype=dtype,
                                                                   test_flags=nat.TEST_INDEX64, **mode))
                assert raw.status == o.status == 0
                if raw.format != "csr":
                    continue  # a COO parse result (stream order) has no index path of its own
                R = oracle_lib.to_raw(o, "csr" if out == nat.OUT_CSR else "parse")
                if raw.indptr.dtype != np.int64 or raw.indices.dtype != np.int64:
                    bad.append((mode, dtype, out, "dtype", raw.indptr.dtype))
                    continue
                if not (np.array_equal(raw.indptr, R.indptr) and np.array_equal(raw.indices, R.indices)
                        and raw.data.tobytes() == R.data.tobytes()):
                    bad.append((mode, dtype, out))
    assert not bad, bad[:4]


@pytest.mark.parametrize("case", ["synth_dense", "synth"])
def test_convert_format_int64_path_equals_oracle(gpu, oracle_lib, monkeypatch, case):
    """convert_format(A, "csr" | "csc") of a COO parse_gfa returns (utils.py:55; cli.py:239 for
    `convert --undirected`) through the int64 index path g2n_coo_to_csr takes past 2^31 - 1 entries
    (TEST_INDEX64 forces it on a small input): int64 indptr / indices holding exactly scipy's values, in
    every COO mode and every CLI dtype; a weighted COO takes the row-band route a weighted COO past
    2^31 - 2 entries takes (three bands here): int64 too, equal values."""
    from gfa2network_amd import _native as nat
    from gfa2network_amd import convert_format, parse_gfa
    from gfa2network_amd import synth

    data = synth.host_bytes(3000, 60000, seed=9) if case == "synth_dense" else _csr_cases()[case]
    bad = []
    for mode in ({"directed": False}, {"asymmetric": True}, {"bidirected": True},
                 {"keep_directed_bidir": True, "asymmetric": True}, {"directed": False, "weight_tag": "RC"}):
        for dtype in ("float64", "float32", "int32", "int8", "bool"):
            monkeypatch.setattr(nat, "TEST_FLAGS", 0)
            A = parse_gfa(io.BytesIO(data), build_graph=False, build_matrix=True, dtype=dtype, **mode)
            assert A.format == "coo"
            o = oracle_lib.run(data, dtype=dtype, **mode)
            R = oracle_lib.to_raw(o, "csr")  # what convert_format(parse_gfa(...), "csr") returns
            Rc = sp.coo_matrix((o.data, (o.rows.astype(np.int32), o.cols.astype(np.int32))),
                               shape=A.shape).tocsc()
            monkeypatch.setattr(nat, "TEST_FLAGS", nat.TEST_INDEX64)
            for fmt, ref in (("csr", R), ("csc", Rc)):
                C = convert_format(A, fmt)
                # every value dtype(1) (no weight tag, or an RC tag absent from every line): the
                # bucket partition's int64 path; other values: the row bands (_coo_to_csr_bands)
                want = np.int64
                if C.indptr.dtype != want or C.indices.dtype != want:
                    bad.append((mode, dtype, fmt, "dtype", C.indptr.dtype))
                if not (np.array_equal(C.indptr, ref.indptr) and np.array_equal(C.indices, ref.indices)
                        and C.data.tobytes() == ref.data.tobytes()):
                    bad.append((mode, dtype, fmt))
    assert not bad, bad[:4]


def test_scan_status_epochs_wrap(gpu, oracle_lib):
    """The single-pass scans reuse their status buffers by epoch (g2n_scan.hip: 4095 epochs, then
    the buffer is cleared): 1500 builds on one context — several scans each, past the wrap on every
    slot — all equal the first and the oracle (a stale word taken as published would shift offsets)."""
    from gfa2network_amd import _native as nat

    data = _canonical_gfa(3, 700, 2500, False, False)
    want = outcome(oracle_run(oracle_lib, data, {"directed": False}, "float64", None))
    first = None
    for i in range(1500):
        raw = nat.build_from_buffer(data, nat.make_options(directed=False, output=nat.OUT_CSR))
        key = (raw.status, raw.indptr.tobytes(), raw.indices.tobytes(), raw.data.tobytes())
        first = first or key
        assert key == first, i
    assert outcome(gpu_run(data, {"directed": False}, "float64", None)) == want


def _band_coo(seed, n, m, dtype, sorted_rows):
    """A COO whose float duplicates sum differently in stream and in sorted order (1e16, 1, -1e16),
    and whose rows below n // 2 are in column order (sorted_rows) while the rest are not."""
    r = np.random.default_rng(seed)
    rows = np.sort(r.integers(0, n, m)).astype(np.int32)
    cols = r.integers(0, n, m).astype(np.int32)
    if sorted_rows:  # the first half of the rows sorted by column inside each row
        lo = rows < n // 2
        order = np.lexsort((cols[lo], rows[lo]))
        cols[lo] = cols[lo][order]
    vals = r.choice(np.array([1e16, 1.0, -1e16, 0.5, 3.0, -2.0]), m)
    dup = r.integers(0, m, m // 4)  # duplicates of existing (row, col) pairs
    rows = np.concatenate([rows, rows[dup]])
    cols = np.concatenate([cols, cols[dup]])
    vals = np.concatenate([vals, r.choice(np.array([1e16, -1e16, 1.0]), len(dup))])
    perm = np.argsort(rows, kind="stable")  # stream order: rows grouped, duplicates later in their row
    return rows[perm], cols[perm], vals[perm].astype(dtype)


@pytest.mark.parametrize("dtype", ["float64", "float32", "int32", "int8", "bool"])
@pytest.mark.parametrize("shape", ["sorted_and_unsorted", "all_sorted", "uniform"])
def test_coo_to_csr_row_bands_equal_scipy(gpu, dtype, shape):
    """The row-band route of convert_format past one call's limit (_coo_to_csr_bands,
    g2n_coo_to_csr_band) on a small COO cut into 2..7 bands: equal to scipy's coo.tocsr() bit for bit —
    including float sums whose order depends on scipy's WHOLE-matrix has_sorted_indices verdict (a
    band sorted on its own is re-run when another band is not) and the uniform partition's bands."""
    from gfa2network_amd import _native as nat

    n = 4000
    rows, cols, vals = _band_coo(5, n, 60000, dtype, shape != "sorted_and_unsorted")
    if shape == "all_sorted":  # every row in column order: scipy sorts nothing
        order = np.lexsort((cols, rows))
        rows, cols, vals = rows[order], cols[order], vals[order]
    if shape == "uniform":
        vals = np.ones(len(rows), dtype=dtype)
    want = sp.coo_matrix((vals, (rows, cols)), shape=(n, n)).tocsr()
    for limit in (len(vals) // 2 + 1, len(vals) // 7 + 1):
        raw = nat.coo_to_csr(rows, cols, vals, n, n, band_entries=limit)
        assert np.array_equal(raw.indptr, want.indptr) and np.array_equal(raw.indices, want.indices), limit
        assert raw.data.tobytes() == want.data.tobytes(), (dtype, shape, limit)
