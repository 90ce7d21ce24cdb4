"""CPU: the product's host+device headers, compiled for the host, against CPython and
libstdc++ themselves.

* pylit.h (the GPU's copy of CPython int()/float() literal semantics) vs int()/float();
* stl_sort.h (the GPU's restatement of libstdc++ std::sort) vs std::sort, including the
  heap-sort fallback the introsort depth limit triggers.
"""
import ctypes
import decimal
import math
import random
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
SRC = ROOT / "tests" / "native" / "hostcheck.cpp"


@pytest.fixture(scope="module")
def hc(tmp_path_factory):
    out = tmp_path_factory.mktemp("hc") / "hostcheck.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", str(out), str(SRC)], check=True)
    lib = ctypes.CDLL(str(out))
    for f in ("hc_py_float", "hc_py_int", "hc_fast_int", "hc_fast_float", "hc_utf8_valid"):
        getattr(lib, f).restype = ctypes.c_int
    lib.hc_sort_both.restype = None
    return lib


def _f(lib, s, transform=1):
    b = s.encode("utf-8", "surrogatepass") if isinstance(s, str) else s
    out = ctypes.c_double()
    r = lib.hc_py_float(b, len(b), ctypes.byref(out))
    return r, out.value


def _i(lib, s, transform=1):
    b = s.encode("utf-8", "surrogatepass") if isinstance(s, str) else s
    out = ctypes.c_double()
    r = lib.hc_py_int(b, len(b), transform, ctypes.byref(out))
    return r, out.value


def ref_float(s):
    try:
        return 1, float(s)
    except ValueError:
        return 0, 0.0


def ref_int(s):
    try:
        v = int(s)
    except ValueError:
        return 0, 0.0
    try:
        return 1, float(v)
    except OverflowError:
        return 2, 0.0


def same(a, b):
    return a[0] == b[0] and (a[0] != 1 or struct.pack("<d", a[1]) == struct.pack("<d", b[1]))


EDGE = ["1", "1.5", "-0.0", "1e400", "nan", "-nan", "NaN", "inf", "-Infinity", "1_0.2_5e-1", "1__0", "_1", "1_",
        ".5", "5.", ".", " 7 ", " 1.25　", "１２.5", "1e", "e5", "+.e1", "0." + "0" * 500 + "1e500",
        "1" * 400 + "e-390", "4.9406564584124654e-324", "2.4703282292062327e-324", "2.4703282292062328e-324",
        "1.7976931348623158e308", "1.7976931348623159e308", "0.1", "0x10", "1e1_0", "1_e5", "in_f", "nAn ", "  ",
        "", "1\x00", "\x0b12\x0c\r", "9007199254740993", "1e-400", "-1e-400", "\x1c1", "٣٤", "1 2",
        "- 5", "+_5", "0" * 5000 + "1", "1" * 4300, "1" * 4301, "9" * 309, " -3 "]


def test_literals_edge_cases(hc):
    for s in EDGE:
        assert same(_f(hc, s), ref_float(s)), s
        assert same(_i(hc, s), ref_int(s)), s


def test_int_bytes_semantics(hc):
    for s in [b" 12 ", b"1_2", b"+12", b"\xd9\xa3", b"12\r", b"12\x00", b"\x1c12", b"", b"6$", b"-0", b"1" * 4301]:
        try:
            int(s)
            ok = 1
        except ValueError:
            ok = 0
        assert (_i(hc, s, transform=0)[0] != 0) == bool(ok), s


def test_literals_fuzz(hc):
    r = random.Random(1)
    for _ in range(100_000):
        k = r.random()
        if k < 0.4:
            s = repr(r.uniform(-1e10, 1e10) * 10 ** r.randint(-300, 300))
        elif k < 0.7:
            digs = "".join(r.choice("0123456789") for _ in range(r.randint(1, 40)))
            p = r.randint(0, len(digs))
            s = digs[:p] + "." + digs[p:] + (f"e{r.randint(-340, 320)}" if r.random() < 0.7 else "")
        else:
            s = "".join(r.choice("0123456789._eE+- \t") for _ in range(r.randint(0, 12)))
        assert same(_f(hc, s), ref_float(s)), s
        assert same(_i(hc, s), ref_int(s)), s


def test_halfway_cases(hc):
    r = random.Random(2)
    for _ in range(5000):
        x = r.uniform(0, 1) * 2.0 ** r.randint(-1074, 1023)
        d = decimal.Decimal(x)
        half = (d + decimal.Decimal(math.nextafter(x, math.inf))) / 2
        for s in (str(half), str(half.next_plus()), str(half.next_minus())):
            assert same(_f(hc, s), ref_float(s)), s


def test_fast_paths_agree_with_python(hc):
    r = random.Random(3)
    for _ in range(50_000):
        s = str(r.randint(-10 ** 15 + 1, 10 ** 15 - 1)) if r.random() < 0.5 else \
            f"{r.randint(0, 10**8)}.{r.randint(0, 10**6)}e{r.randint(-15, 15)}"
        b = s.encode()
        out = ctypes.c_double()
        fn = hc.hc_fast_int if "." not in s else hc.hc_fast_float
        if fn(b, len(b), ctypes.byref(out)):
            want = float(int(s)) if "." not in s else float(s)
            assert struct.pack("<d", out.value) == struct.pack("<d", want), s


def test_utf8_validation(hc):
    r = random.Random(4)
    for _ in range(20000):
        b = bytes(r.randint(0, 255) if r.random() < 0.3 else r.randint(0x80, 0xBF) for _ in range(r.randint(0, 6)))
        try:
            b.decode()
            ok = 1
        except UnicodeDecodeError:
            ok = 0
        assert hc.hc_utf8_valid(b, len(b)) == ok, b


def _sort_both(hc, keys):
    keys = np.ascontiguousarray(keys, dtype=np.int32)
    a = np.zeros(len(keys), np.int32)
    b = np.zeros(len(keys), np.int32)
    hc.hc_sort_both(keys.ctypes.data_as(ctypes.c_void_p), len(keys), a.ctypes.data_as(ctypes.c_void_p),
                    b.ctypes.data_as(ctypes.c_void_p))
    return a, b


def test_stl_sort_random(hc):
    r = random.Random(5)
    for trial in range(2000):
        n = r.randint(0, 400)
        kmax = r.choice([1, 2, 3, 5, 10, 50, 1000])
        keys = np.array([r.randint(0, kmax) for _ in range(n)], dtype=np.int32)
        if trial % 7 == 0:
            keys.sort()
        if trial % 11 == 0:
            keys = keys[::-1].copy()
        a, b = _sort_both(hc, keys)
        assert np.array_equal(a, b), trial


def test_stl_sort_depth_limit_fallback(hc):
    """Median-of-3 killer sequences drive introsort into its heap-sort fallback."""
    for n in (64, 257, 1000, 4096):
        k = n // 2
        keys = np.empty(n, np.int32)
        for i in range(1, k + 1):  # Musser's median-of-3 killer
            if i % 2:
                keys[i - 1] = i
                keys[i] = k + i
            keys[k + i - 1] = 2 * i
        a, b = _sort_both(hc, keys)
        assert np.array_equal(a, b)
        organ = np.concatenate([np.arange(n // 2), np.arange(n // 2)[::-1]]).astype(np.int32)
        a, b = _sort_both(hc, organ)
        assert np.array_equal(a, b)
