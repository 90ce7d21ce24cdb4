"""Golden stderr of the reference's verbose convert_format / save_matrix (gfa2network/utils.py:40-105)
with tqdm importable (tqdm draws the progress line: utils.py:8-14, 49-51, 56-59, 78-80, 99-102).

Runs in the build container with /root/reference importable; writes
tests/golden/expected/verbose.json: per case the captured stderr with the elapsed-time field
normalised ("MM:SS" -> "<T>"), the output file's suffix, and the exception (type, message) if any.
"""
import contextlib
import io
import json
import re
import sys
import tempfile
from pathlib import Path

import numpy as np
import scipy.sparse as sp

OUT = Path(__file__).parent / "expected" / "verbose.json"


def norm(s: str) -> str:
    s = re.sub(r"\d\d:\d\d(:\d\d)?", "<T>", s)
    return re.sub(r"done in [\d,]+\.\ds", "done in <S>s", s)


def matrix():
    rows = np.array([0, 1, 2, 2, 0], dtype=np.int32)
    cols = np.array([1, 2, 0, 0, 1], dtype=np.int32)
    return sp.coo_matrix((np.ones(5), (rows, cols)), shape=(3, 3))


def cases():
    A = matrix()
    out = []
    for fmt in ("csr", "csc", "dok", "coo", "CSR", "bsr"):
        out.append(("convert", fmt, "coo"))
        out.append(("convert", fmt, "csr"))
    for suffix in (".npz", ".npy", ".csv", ".txt"):
        out.append(("save", suffix, "csr"))
    out.append(("save_guard", ".npy", "csr"))
    return A, out


def run(impl_convert, impl_save, tmpdir):
    A, cs = cases()
    res = []
    for kind, arg, src in cs:
        M = A if src == "coo" else A.tocsr()
        err = io.StringIO()
        exc = None
        with contextlib.redirect_stderr(err):
            try:
                if kind == "convert":
                    impl_convert(M, arg, verbose=True)
                elif kind == "save":
                    impl_save(M, Path(tmpdir) / f"m{arg}", verbose=True)
                else:
                    impl_save(M, Path(tmpdir) / f"m{arg}", verbose=True, max_dense_gb=1e-12)
            except Exception as e:  # noqa: BLE001 - recorded
                exc = [type(e).__name__, str(e).replace(str(tmpdir), "<DIR>")]
        res.append({"kind": kind, "arg": arg, "src": src,
                    "stderr": norm(err.getvalue().replace(str(tmpdir), "<DIR>")), "exc": exc})
    return res


if __name__ == "__main__":
    sys.path.insert(0, "/root/reference")  # the reference, in the build container only
    from gfa2network import utils

    assert utils._HAS_TQDM, "the golden needs tqdm importable"
    with tempfile.TemporaryDirectory() as d:
        OUT.write_text(json.dumps(run(utils.convert_format, utils.save_matrix, d), indent=1, ensure_ascii=False))
    print(f"wrote {OUT}")
