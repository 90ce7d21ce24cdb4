"""The direct-address dictionary tier on the lean front end (k_tile_lean kLeanDirClaim /
kLeanDirEdges): inputs whose S lines come first and whose segment names are one common prefix
(possibly empty), a decimal and one common suffix without digits (possibly empty) — the decimal
canonical, or zero-padded to one width — decimal ids out of S order, minigraph's "s<n>", hifiasm's
"utg000123l" —
take a plain array as the dictionary (S line k claims direct[v] = k; an edge name is one random
4-byte read).  builders.py:190-198: with every S line first and no repeated name, a key's first
touch is its S line, so node id = S index.  Every case is compared with the oracle, with the lean
hash tier (TEST_NO_DIRECT) and with the classic tiers (TEST_NO_HASH_LEAN); cases that break the
premise (a repeated value, a value past the table, another prefix, leading zeros, "0", 11 digits,
an edge key no S line names, an S line after an edge line, unsupported or malformed records) must
fall back and still match.
"""
import random

import pytest

from test_gpu_diff import gpu_run, oracle_run, outcome

pytestmark = pytest.mark.gpu

MODES = [{}, {"directed": False}, {"asymmetric": True}]


def _gfa(seed, n_s, n_l, prefix="", spread=1, ov="0M", fmt=None, in_order=False):
    r = random.Random(seed)
    vals = list(range(1, n_s + 1)) if in_order else r.sample(range(1, spread * n_s + 1), n_s)  # distinct values
    names = [fmt % v if fmt else f"{prefix}{v}" for v in vals]
    lines = [f"S\t{k}\t{'ACGT' * r.randint(0, 3)}\n" for k in names]
    for _ in range(n_l):
        a = r.randrange(n_s)
        b = min(n_s - 1, a + r.randint(0, 5))
        lines.append(f"L\t{names[a]}\t{r.choice('+-')}\t{names[b]}\t{r.choice('+-')}\t{ov}\n")
    return names, lines


def _case(name):
    names, L = _gfa(21, 6000, 30000)
    n = 6000
    if name == "permuted":
        return L, True
    if name == "prefix_s":
        return _gfa(22, 6000, 30000, prefix="s")[1], True
    if name == "prefix_8_bytes_gaps":  # values up to 3 x the S lines: inside the 4 x table
        return _gfa(23, 6000, 30000, prefix="node_id_", spread=3)[1], True
    if name == "hifiasm_utg_in_order":  # zero-padded, common suffix: "utg000001l", ...
        return _gfa(25, 6000, 30000, fmt="utg%06dl", in_order=True)[1], True
    if name == "zero_padded_shuffled":
        return _gfa(26, 6000, 30000, fmt="node%07d", spread=3)[1], True
    if name == "canonical_with_suffix":
        return _gfa(27, 6000, 30000, fmt="ctg%dc")[1], True
    if name == "width_break":  # one name one digit wider: value 77 twice (the width keeps names apart)
        _, L2 = _gfa(28, 6000, 30000, fmt="utg%06dl", in_order=True)
        return L2[:50] + ["S\tutg0000077l\t*\n"] + L2[50:], False
    if name == "suffix_break":
        _, L2 = _gfa(29, 6000, 30000, fmt="utg%06dl", in_order=True)
        return L2[:50] + ["S\tutg999999c\t*\n"] + L2[50:], False
    if name == "suffix_with_digit":  # the first name's suffix holds a digit: no pattern
        return _gfa(30, 6000, 30000, fmt="tig%da1")[1], False
    if name == "padded_edge_unpadded":  # an edge names "utg77l" (unpadded): not a defined name
        _, L2 = _gfa(31, 6000, 30000, fmt="utg%06dl", in_order=True)
        return L2[:7000] + ["L\tutg77l\t+\tutg000003l\t-\t0M\n"] + L2[7000:], False
    if name == "ten_digit_values":
        _, L2 = _gfa(24, 3000, 12000)
        return [ln.replace("S\t", "S\t10000", 1) if ln.startswith("S") else
                ln.replace("L\t", "L\t10000", 1).replace("\t+\t", "\t+\t10000", 1).replace("\t-\t", "\t-\t10000", 1)
                for ln in L2], False  # (values past the table: the hash tiers)
    if name == "p_and_header_lines":
        return ["H\tVN:Z:1.0\n"] + L[:n] + ["P\tp1\t" + names[0] + "+," + names[1] + "-\t*\n"] + L[n:], True
    if name == "repeated_value":
        return L[:n] + ["S\t" + names[77] + "\tAC\n"] + L[n:], False
    if name == "other_prefix":
        return L[:50] + ["S\tx5000000\t*\n"] + L[50:], False
    if name == "leading_zero":
        return L[:50] + ["S\t0777777\t*\n"] + L[50:], False
    if name == "zero":
        return L[:50] + ["S\t0\t*\n"] + L[50:], False
    if name == "eleven_digits":
        return L[:50] + ["S\t12345678901\t*\n"] + L[50:], False
    if name == "value_past_table":
        return L[:50] + ["S\t99999999\t*\n"] + L[50:], False
    if name == "s_after_edges":
        return L[:100] + L[n:n + 100] + L[100:n] + L[n + 100:], False
    if name == "edge_to_undefined_value":
        return L[:7000] + ["L\t999999\t+\t" + names[3] + "\t-\t0M\n"] + L[7000:], False
    if name == "edge_to_non_decimal":
        return L[:7000] + ["L\tnobody\t+\t" + names[3] + "\t-\t0M\n"] + L[7000:], False
    if name == "unsupported_record":
        return L[:7000] + ["W\tsample\t1\tchr1\t0\t10\t>x\n"] + L[7000:], False
    if name == "malformed_link":
        return L[:7000] + ["L\t" + names[1] + "\t+\n"] + L[7000:], False
    # the passes' tile lists (k_tile_lists): no edge line at all; tiles holding only P lines at the
    # end (claim list, no edge list); an S line in a tile far past the edge-only tiles
    if name == "s_lines_only":
        return L[:n], True
    if name == "p_only_tiles_at_end":
        return L + ["P\tp%d\t%s+,%s-\t*\n" % (i, names[i], names[i + 1]) for i in range(4000)], True
    if name == "s_line_in_a_late_tile":
        return L + ["S\t%d\tAC\n" % (n + 1)] + L[n:n + 3000], False
    raise KeyError(name)


CASES = ["permuted", "prefix_s", "prefix_8_bytes_gaps", "hifiasm_utg_in_order", "zero_padded_shuffled",
         "canonical_with_suffix", "width_break", "suffix_break", "suffix_with_digit", "padded_edge_unpadded",
         "ten_digit_values", "p_and_header_lines", "repeated_value",
         "other_prefix", "leading_zero", "zero", "eleven_digits", "value_past_table", "s_after_edges",
         "edge_to_undefined_value", "edge_to_non_decimal", "unsupported_record", "malformed_link",
         "s_lines_only", "p_only_tiles_at_end", "s_line_in_a_late_tile"]


@pytest.mark.parametrize("case", CASES)
def test_direct_tier_equals_oracle_and_other_tiers(gpu, oracle_lib, monkeypatch, case):
    from gfa2network_amd import _native as nat

    lines, eligible = _case(case)
    data = "".join(lines).encode()
    for mode in MODES:
        raw = nat.build_from_buffer(data, nat.make_options(**mode))
        ph = raw.phase_ms
        took = "direct_lookup" in ph and "insert_lookup" not in ph and "parse" not in ph
        if raw.status == 0:
            assert took == eligible, (case, mode, sorted(ph))
        for dtype in ("float64", "int8", "bool"):
            a = outcome(gpu_run(data, mode, dtype, None))
            assert a == outcome(oracle_run(oracle_lib, data, mode, dtype, None)), (case, mode, dtype)
            for flags, what in ((nat.TEST_NO_DIRECT, "lean hash"), (nat.TEST_NO_HASH_LEAN, "classic")):
                monkeypatch.setattr(nat, "TEST_FLAGS", flags)
                assert a == outcome(gpu_run(data, mode, dtype, None)), (case, mode, dtype, what)
                monkeypatch.setattr(nat, "TEST_FLAGS", 0)


def test_direct_tier_on_ids_in_order(gpu, oracle_lib, monkeypatch):
    """TEST_DICT_DIRECT: decimal ids "1".."N" in S order through the direct tier instead of the
    decimal-id parse — same answer, every mode family."""
    from gfa2network_amd import _native as nat
    from gfa2network_amd import synth

    data = synth.host_bytes(30_000, 120_000, seed=8)
    for mode in MODES:
        want = outcome(gpu_run(data, mode, "float64", None))
        monkeypatch.setattr(nat, "TEST_FLAGS", nat.TEST_DICT_DIRECT)
        raw = nat.build_from_buffer(data, nat.make_options(**mode))
        assert "direct_lookup" in raw.phase_ms, sorted(raw.phase_ms)
        assert outcome(gpu_run(data, mode, "float64", None)) == want, mode
        monkeypatch.setattr(nat, "TEST_FLAGS", 0)
        assert want == outcome(oracle_run(oracle_lib, data, mode, "float64", None)), mode


def test_direct_tier_synthetic_large_equals_lean_hash(gpu, monkeypatch):
    """10^7 edges of the generator with permuted decimal names (names="permuted"): the direct tier
    against the lean hash tier, bit for bit, CSR and COO outputs, names included."""
    from gfa2network_amd import _native as nat
    from gfa2network_amd import synth

    data = synth.host_bytes(2_000_000, 8_000_000, seed=5, names="permuted")
    for mode in ({}, {"directed": False}):
        raw = nat.build_from_buffer(data, nat.make_options(**mode))
        assert raw.status == 0 and "direct_lookup" in raw.phase_ms and "parse" not in raw.phase_ms, sorted(raw.phase_ms)
        a = outcome(gpu_run(data, mode, "float64", None))
        monkeypatch.setattr(nat, "TEST_FLAGS", nat.TEST_NO_DIRECT)
        b = outcome(gpu_run(data, mode, "float64", None))
        monkeypatch.setattr(nat, "TEST_FLAGS", 0)
        assert a == b, mode


# ---- the extended tile-local lean parse: bidirected keys and one integer weight tag (round 5) ----
def _ext_case(name):
    r = random.Random(31)
    n_s, n_l = 3000, 12000
    S = [f"S\t{k}\t{'ACGT' * r.randint(0, 2)}\n" for k in range(1, n_s + 1)]

    def link(tag=True):
        a = r.randint(1, n_s)
        b = min(n_s, a + r.randint(0, 4))
        t = f"\tRC:i:{r.randint(-50, 99)}" if tag and r.random() < 0.9 else ""
        return f"L\t{a}\t{r.choice('+-')}\t{b}\t{r.choice('+-')}\t0M{t}\n"
    L = [link() for _ in range(n_l)]
    if name == "canonical":
        return S + L, True
    if name == "no_tags":
        return S + [link(False) for _ in range(n_l)], True
    if name == "zero_and_negative":
        return S + L[:100] + ["L\t1\t+\t2\t-\t0M\tRC:i:0\n", "L\t2\t-\t3\t-\t0M\tRC:i:-7\n"] + L[100:], True
    if name == "leading_zero_value":  # int("007") == 7: the full parse decides, same answer
        return S + L[:100] + ["L\t1\t+\t2\t-\t0M\tRC:i:007\n"] + L[100:], False
    if name == "plus_sign":
        return S + L[:100] + ["L\t1\t+\t2\t-\t0M\tRC:i:+5\n"] + L[100:], False
    if name == "float_type":
        return S + L[:100] + ["L\t1\t+\t2\t-\t0M\tRC:f:1.5\n"] + L[100:], False
    if name == "other_tag":
        return S + L[:100] + ["L\t1\t+\t2\t-\t0M\tID:Z:x\n"] + L[100:], False
    if name == "two_tags":
        return S + L[:100] + ["L\t1\t+\t2\t-\t0M\tRC:i:3\tRC:i:4\n"] + L[100:], False
    if name == "ten_digits":
        return S + L[:100] + ["L\t1\t+\t2\t-\t0M\tRC:i:1234567890\n"] + L[100:], False
    if name == "bad_orientation":
        return S + L[:100] + ["L\t1\t*\t2\t-\t0M\n"] + L[100:], False
    raise KeyError(name)


TAG_ONLY = {"leading_zero_value", "plus_sign", "float_type", "other_tag", "two_tags", "ten_digits"}
EXT_CASES = ["canonical", "no_tags", "zero_and_negative", "leading_zero_value", "plus_sign", "float_type",
             "other_tag", "two_tags", "ten_digits", "bad_orientation"]
EXT_MODES = [({"bidirected": True}, None), ({"bidirected": True}, "RC"), ({"bidirected": True, "keep_directed_bidir": True}, "RC"),
             ({}, "RC"), ({"directed": False}, "RC"), ({"asymmetric": True}, "RC")]


@pytest.mark.parametrize("case", EXT_CASES)
def test_extended_lean_parse_equals_oracle(gpu, oracle_lib, monkeypatch, case):
    """Decimal-id files built bidirected and / or with a weight tag take the extended tile-local lean
    parse (no K1, no full parse): "name:o" keys 2k / 2k + 1, the reverse twins (builders.py:211-234) and
    the tag's canonical integer value (parser.py:179-204); other spellings fall back to the full parse.
    Every mode x dtype equals the oracle and the K1 + lean-parse path (TEST_NO_EXT_LEAN)."""
    from gfa2network_amd import _native as nat

    lines, eligible = _ext_case(case)
    data = "".join(lines).encode()
    for mode, wt in EXT_MODES:
        raw = nat.build_from_buffer(data, nat.make_options(weight_tag=wt, **mode))
        if raw.status == 0 and (wt or mode.get("bidirected")):
            took = "tiles" not in raw.phase_ms and "parse" in raw.phase_ms
            # (a tag the lean parse refuses matters only when the build reads that tag)
            want = eligible or (wt is None and case in TAG_ONLY)
            assert took == want, (case, mode, wt, sorted(raw.phase_ms))
        for dtype in ("float64", "float32", "int8", "bool"):
            a = outcome(gpu_run(data, mode, dtype, wt))
            assert a == outcome(oracle_run(oracle_lib, data, mode, dtype, wt)), (case, mode, wt, dtype)
            monkeypatch.setattr(nat, "TEST_FLAGS", nat.TEST_NO_EXT_LEAN)
            assert a == outcome(gpu_run(data, mode, dtype, wt)), (case, mode, wt, dtype, "K1 path")
            monkeypatch.setattr(nat, "TEST_FLAGS", 0)


# ---- bidirected / weighted builds on the lean hash and direct tiers (round 5) ----
def _ext_tier_case(name):
    r = random.Random(sum(name.encode()))
    n_s = 3000
    if name.startswith("permuted"):
        names = [str(v) for v in r.sample(range(1, n_s + 1), n_s)]
    else:
        seen = set()
        while len(seen) < n_s:
            seen.add("ctg_%08x" % r.getrandbits(32))
        names = sorted(seen, key=lambda _: r.random())
    S = [f"S\t{k}\t{'ACGT' * r.randint(0, 2)}\n" for k in names]

    def link(tag=True):
        a = r.randrange(n_s)
        b = min(n_s - 1, a + r.randint(0, 4))
        t = f"\tRC:i:{r.randint(-50, 99)}" if tag and r.random() < 0.9 else ""
        return f"L\t{names[a]}\t{r.choice('+-')}\t{names[b]}\t{r.choice('+-')}\t0M{t}\n"
    L = [link() for _ in range(12000)]
    tier = "direct_lookup" if name.startswith("permuted") else "insert_lookup"
    if name in ("permuted", "hashed"):
        return S + L, tier
    if name in ("permuted_float_tag", "hashed_float_tag"):
        return S + L[:100] + [f"L\t{names[1]}\t+\t{names[2]}\t-\t0M\tRC:f:1.5\n"] + L[100:], None
    if name == "hashed_two_tags":
        return S + L[:100] + [f"L\t{names[1]}\t+\t{names[2]}\t-\t0M\tRC:i:3\tRC:i:4\n"] + L[100:], None
    if name == "hashed_no_tags":
        return S + [link(False) for _ in range(12000)], tier
    raise KeyError(name)


EXT_TIER_CASES = ["permuted", "hashed", "permuted_float_tag", "hashed_float_tag", "hashed_two_tags", "hashed_no_tags"]


@pytest.mark.parametrize("case", EXT_TIER_CASES)
def test_extended_lean_tiers_equal_oracle(gpu, oracle_lib, monkeypatch, case):
    """Names that are not the decimal ids, built bidirected and / or with a weight tag: the direct and
    lean hash tiers' edge passes in their extended instance ("name:o" ids 2i + o and the reverse
    twins, one canonical integer tag per edge; builders.py:199-234, parser.py:179-204).  Every mode x
    dtype equals the oracle and the classic tiers (TEST_NO_HASH_LEAN); a tag the lean shape refuses
    sends the build to the full parse when the build reads that tag."""
    from gfa2network_amd import _native as nat

    lines, tier = _ext_tier_case(case)
    data = "".join(lines).encode()
    for mode, wt in EXT_MODES:
        raw = nat.build_from_buffer(data, nat.make_options(weight_tag=wt, **mode))
        if raw.status == 0:
            ph = raw.phase_ms  # (a failed lean pass leaves its phase, then the full parse runs)
            took = (None if "parse" in ph else "insert_lookup" if "insert_lookup" in ph else
                    "direct_lookup" if "direct_lookup" in ph else None)
            want = tier if (tier or wt is None) else None
            if want is None and wt is None:
                want = "direct_lookup" if case.startswith("permuted") else "insert_lookup"
            assert took == want, (case, mode, wt, sorted(ph))
        for dtype in ("float64", "float32", "int8", "bool"):
            a = outcome(gpu_run(data, mode, dtype, wt))
            assert a == outcome(oracle_run(oracle_lib, data, mode, dtype, wt)), (case, mode, wt, dtype)
            monkeypatch.setattr(nat, "TEST_FLAGS", nat.TEST_NO_HASH_LEAN)
            assert a == outcome(gpu_run(data, mode, dtype, wt)), (case, mode, wt, dtype, "classic")
            monkeypatch.setattr(nat, "TEST_FLAGS", 0)


# ---- the decimal-id layout behind one constant prefix (round 6: minigraph's "s1".."sN" in S order) ----
def _prefixed_case(name):
    r = random.Random(41)
    n_s, n_l = 5000, 20000

    def gfa(pre, rc=False, n=n_s):
        S = [f"S\t{pre}{k}\t{'ACGT' * r.randint(0, 3)}\n" for k in range(1, n + 1)]
        L = []
        for _ in range(n_l):
            a = r.randint(1, n)
            b = min(n, a + r.randint(0, 5))
            t = f"\tRC:i:{r.randint(-9, 99)}" if rc else ""
            L.append(f"L\t{pre}{a}\t{r.choice('+-')}\t{pre}{b}\t{r.choice('+-')}\t0M{t}\n")
        return S, L
    if name == "s_in_order":
        S, L = gfa("s")
        return S + L, True
    if name == "eight_byte_prefix":
        S, L = gfa("node_id_")
        return S + L, True
    if name == "nine_byte_prefix":  # longer than the layout takes: the hash tiers
        S, L = gfa("contig_id")
        return S + L, False
    if name == "weights_and_header":
        S, L = gfa("s", rc=True)
        return ["H\tVN:Z:1.0\n"] + S + L, True
    if name == "edge_without_prefix":
        S, L = gfa("s")
        return S + L[:500] + ["L\t7\t+\ts8\t-\t0M\n"] + L[500:], False
    if name == "s_without_prefix":
        S, L = gfa("s")
        return S[:40] + ["S\t41\t*\n"] + S[41:] + L, False
    if name == "leading_zero":
        S, L = gfa("s")
        return S + L[:500] + ["L\ts07\t+\ts8\t-\t0M\n"] + L[500:], False
    if name == "empty_decimal":
        S, L = gfa("s")
        return S + L[:500] + ["L\ts\t+\ts8\t-\t0M\n"] + L[500:], False
    if name == "other_prefix":
        S, L = gfa("s")
        return S[:40] + ["S\tt41\t*\n"] + S[41:] + L, False
    if name == "past_the_segments":
        S, L = gfa("s")
        return S + L[:500] + [f"L\ts{n_s + 3}\t+\ts8\t-\t0M\n"] + L[500:], False
    if name == "repeated_name":
        S, L = gfa("s")
        return S + ["S\ts77\t*\n"] + L, False
    if name == "out_of_order":
        S, L = gfa("s")
        return S[:10] + [S[11], S[10]] + S[12:] + L, False
    if name == "s_after_edges":
        S, L = gfa("s")
        return S[:-5] + L[:100] + S[-5:] + L[100:], False
    raise KeyError(name)


PREFIXED = ["s_in_order", "eight_byte_prefix", "nine_byte_prefix", "weights_and_header", "edge_without_prefix",
            "s_without_prefix", "leading_zero", "empty_decimal", "other_prefix", "past_the_segments",
            "repeated_name", "out_of_order", "s_after_edges"]


@pytest.mark.parametrize("case", PREFIXED)
def test_prefixed_decimal_layout_equals_oracle(gpu, oracle_lib, monkeypatch, case):
    """Names P + str(k + 1) in S order (P: 1-8 bytes without a digit): the tile-local decimal-id parse
    strips P (ParseOpts::dpre; names P + str(k + 1) by arithmetic) — no K1, no dictionary.  Against
    the oracle and against the direct / hash tiers (TEST_NO_DEC_PREFIX), every mode family, bidirected
    and weighted builds (the extended instance); premise breaks fall back with the same answer."""
    from gfa2network_amd import _native as nat

    lines, eligible = _prefixed_case(case)
    data = "".join(lines).encode()
    wt = "RC" if case == "weights_and_header" else None
    for mode in MODES + [{"bidirected": True}, {"bidirected": True, "directed": False}]:
        raw = nat.build_from_buffer(data, nat.make_options(weight_tag=wt, **mode))
        ph = raw.phase_ms
        took = not any(k in ph for k in ("tiles", "direct_lookup", "insert_lookup", "insert_claim"))
        if raw.status == 0:
            assert took == eligible, (case, mode, sorted(ph))
        for dtype in ("float64", "int8"):
            a = outcome(gpu_run(data, mode, dtype, wt))
            assert a == outcome(oracle_run(oracle_lib, data, mode, dtype, wt)), (case, mode, dtype)
            monkeypatch.setattr(nat, "TEST_FLAGS", nat.TEST_NO_DEC_PREFIX)
            assert a == outcome(gpu_run(data, mode, dtype, wt)), (case, mode, dtype, "direct / hash tiers")
            monkeypatch.setattr(nat, "TEST_FLAGS", 0)


def test_prefixed_decimal_export_equals_oracle(gpu, oracle_lib):
    """export --format edge-list of a prefixed build: the names come from the blob (the arithmetic
    render knows only the bare decimals) — the oracle's bytes."""
    from gfa2network_amd import _native as nat

    data = "".join(_prefixed_case("s_in_order")[0]).encode()
    for bidir in (False, True):
        raw = nat.build_from_buffer(data, nat.make_options(bidirected=bidir, output=nat.OUT_EDGE_LIST))
        want, err, _ = oracle_lib.export_edge_list(data, bidirected=bidir)
        assert err is None and raw.status == 0 and bytes(raw.data) == want, bidir
