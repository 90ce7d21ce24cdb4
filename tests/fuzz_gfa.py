"""Random GFA texts that stress the parse rules of SURVEY.md Appendix A.

Deterministic per seed.  Mixes well-formed GFA-1 / GFA-2 records with the quirks the
reference's parser has (CR kept, GFA2-style L, E/C coordinate heuristics, arbitrary
orientation strings, duplicate / malformed / non-UTF-8 tags, unknown and blank lines,
names containing '+', '-' and ':'), so GPU-vs-oracle comparisons cover them.
"""
from __future__ import annotations

import random

NAME_POOL = ["a", "b", "c", "a+", "b-", "x:+", "1", "2", "10", "é", "日本", "n_1", "+", "-", "", "s1", "s2"]
ORIS = ["+", "-", "+", "-", "+\r", "x", "", "+:x", "\xff"]
INTS = ["0", "1", "-3", "7", "+12", " 4 ", "1_0", "99999999999999999999", "٣", "1__0", "", "x", "9" * 320]
FLOATS = ["1.5", "-0.0", "nan", "-nan", "inf", "1e400", "1e-400", ".5", "5.", "1_0.5", "0.1", "2.2250738585072011e-308",
          "1.7976931348623159e308", "3.4028236e38", "1e", "abc", "1.0000000000000002", "123456789012345678901234567890"]


def _name(r: random.Random) -> str:
    if r.random() < 0.7:
        return str(r.randint(1, 12))
    return r.choice(NAME_POOL)


def _tag(r: random.Random, wt: str) -> str:
    key = wt if r.random() < 0.7 else r.choice(["XX", "rc", "RC", ""])
    k = r.random()
    if k < 0.4:
        return f"{key}:i:{r.choice(INTS)}"
    if k < 0.75:
        return f"{key}:f:{r.choice(FLOATS)}"
    if k < 0.85:
        return f"{key}:Z:{r.choice(['x', '1', ''])}"
    if k < 0.9:
        return f"{key}:B:1,2"
    return r.choice(["RC", "RC:i", "::", "RC::3"])


def _line(r: random.Random, wt: str, allow_errors: bool) -> bytes:
    k = r.random()
    tags = "".join("\t" + _tag(r, wt) for _ in range(r.choice([0, 0, 1, 1, 2])))
    if k < 0.25:
        seq = r.choice(["*", "ACGT", "4", "10"])
        return f"S\t{_name(r)}\t{seq}{tags}\n".encode()
    if k < 0.65:
        u, v = _name(r), _name(r)
        o1, o2 = r.choice("+-"), r.choice(ORIS)
        if r.random() < 0.15:  # GFA2-style L: orientations embedded in the names
            return f"L\t{u}{r.choice(['+', '-', ''])}\t{v}{r.choice(['+', '-'])}\t*{tags}\n".encode("utf-8", "surrogateescape")
        line = f"L\t{u}\t{o1}\t{v}\t{o2}\t{r.choice(['0M', '*'])}{tags}"
        return (line + r.choice(["\n", "\n", "\r\n"])).encode("utf-8", "surrogateescape").replace(b"\xc3\xbf", b"\xff")
    if k < 0.72:
        u, v = _name(r), _name(r)
        if r.random() < 0.5:
            c = [r.choice(["0", "6", "6$", " 1", "x"]) for _ in range(4)]
            return f"E\t*\t{u}{r.choice('+-')}\t{v}{r.choice('+-')}\t{c[0]}\t{c[1]}\t{c[2]}\t{c[3]}\t6M{tags}\n".encode()
        return f"E\t*\t{u}\t{r.choice('+-')}\t{v}\t{r.choice('+-')}{tags}\n".encode()
    if k < 0.77:
        u, v = _name(r), _name(r)
        return f"C\t{u}\t{r.choice('+-')}\t{v}\t{r.choice('+-')}\t1\t5M{tags}\n".encode()
    if k < 0.82:
        return r.choice([b"P\tp\ta+,b-\t*\n", b"O\to\ta+ b-\n", b"H\tVN:Z:1.0\n", b"F\tx\n", b"Sx\tq\n"])
    if k < 0.86:
        return r.choice([b"#comment\n", b"\n", b"W\tx\n", b"\r\n"])
    if allow_errors and k < 0.875:
        return r.choice([b"L\ta\t+\tb\n", b"S\n", b"P\tp\n", b"E\t1\t2\n", b"L\t\tb\t*\t*\n", b"\xfejunk\n",
                         b"L\ta\t+\tb\t\xfe\t*\n"])
    return f"L\t{_name(r)}\t+\t{_name(r)}\t-\t*{tags}\n".encode()


def make(seed: int, n_lines: int = 60, allow_errors: bool = True, wt: str = "RC") -> bytes:
    r = random.Random(seed)
    out = b"".join(_line(r, wt, allow_errors) for _ in range(n_lines))
    if r.random() < 0.2 and out.endswith(b"\n"):
        out = out[:-1]  # last line without newline
    return out
