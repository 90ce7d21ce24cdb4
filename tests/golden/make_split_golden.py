#!/usr/bin/env python3
"""Golden fixtures for ``parse_gfa(..., split_on_alignment=True)`` (builders.py:110-128 ->
_parse_gfa_split, builders.py:302-568), from the REAL reference.

Runs ONLY in the build container, where the pure-Python reference is importable from
/root/reference.  Writes the hand-written split inputs to tests/golden/inputs_split/ and, for
those plus every input under tests/golden/inputs/, per flag mode, the returned matrix (format,
shape, dtype, arrays), the node list, the RuntimeWarnings and the exception to
tests/golden/expected/split.json (plain data; arrays base64).
"""
from __future__ import annotations

import base64
import json
import sys
import warnings
from pathlib import Path

REF = "/root/reference"
HERE = Path(__file__).resolve().parent
INPUTS = HERE / "inputs_split"
MODES = {
    "default": {}, "undirected": {"directed": False}, "asym": {"asymmetric": True},
    "bidir": {"bidirected": True}, "bidir_keep": {"bidirected": True, "keep_directed_bidir": True},
    "bidir_undirected_rc": {"bidirected": True, "directed": False, "weight_tag": "RC"},
    "rc_int8": {"weight_tag": "RC", "dtype": "int8"}, "strip_raw": {"strip_orientation": True, "raw_bytes_id": True},
}

SPLIT = {
    # the reference's GFA2 layout (parser.py:254-288): E id u[+-] from_s from_e v[+-] to_s to_e cigar [tags]
    "e_coords": "S\ta\t10\tACGTACGTAC\nS\tb\t8\t*\nS\tc\t*\n"
                "E\te1\ta+\t2\t6\tb-\t0\t4\t4M\tRC:i:3\nE\te2\ta+\t0\t10\tc+\t0\t3\t*\n"
                "L\ta\t+\tb\t-\t0M\tRC:i:7\nL\tb\t-\tc\t+\t*\n",
    "c_records": "S\tr\t20\t*\nS\tq\t12\t*\nC\tr\t+\tq\t-\t5\t3M\nC\tx\tr+\t3\t15\tq-\t1\t8\t*\tRC:i:2\n"
                 "C\ty\tr-\t0\t20\tq+\t0\t12\t*\n",
    "e_fallback": "S\t1\t5\t*\nS\t2\t7\t*\nE\t*\t1\t+\t2\t-\tRC:i:4\nE\te\t1+\tx\t3\t2-\t0\t2\t*\n",
    "no_length_segments": "S\tu\t*\nS\tv\tACGT\nE\te\tu+\t1\t3\tv+\t2\t2\t*\nE\tf\tu-\t3\t5\tv+\t0\t1\t*\n"
                          "L\tu\t+\tv\t+\t0M\n",
    "dup_segments": "S\ts\t10\t*\nS\tt\t4\t*\nS\ts\t6\t*\nE\te\ts+\t0\t6\tt+\t0\t4\t*\n"
                    "E\tf\ts+\t0\t10\tt+\t0\t4\t*\nL\ts\t+\tt\t-\t0M\n",
    "e_before_s": "E\te\tm+\t2\t4\tn+\t1\t3\t*\nS\tm\t6\t*\nS\tn\t5\t*\nL\tn\t+\tm\t+\t0M\n",
    "missing_segments": "S\ta\t4\t*\nE\te\ta+\t0\t2\tzz+\t0\t1\t*\nE\tf\tyy+\t0\t2\ta+\t0\t1\t*\n"
                        "E\tg\ta+\t1\t3\ta+\t0\t2\t*\nL\ta\t+\tww\t-\t0M\nL\tvv\t+\ta\t-\t0M\n"
                        "E\th\ta+\t0\t4\ta-\t0\t4\t*\n",
    "missing_nonutf8": "S\ta\t4\t*\nL\ta\t+\tb\xff\t-\t0M\n",
    "coords_out_of_range": "S\tk\t5\t*\nS\tl\t5\t*\nE\te\tk+\t-3\t2\tl+\t4\t9\t*\nE\tf\tk+\t-3\t0\tl-\t9\t12\t*\n",
    "many_nodes": "S\tg\t100\t*\nS\th\t100\t*\n" + "".join(
        f"E\te{i}\tg+\t{i}\t{i + 1}\th+\t{2 * i}\t{2 * i + 1}\t*\n" for i in range(0, 60, 2)),
    "full_with_interior": "S\tp\t9\t*\nS\tq\t9\t*\nE\te\tp+\t3\t5\tq+\t0\t9\t*\nE\tf\tp+\t0\t9\tq-\t0\t9\t*\n"
                          "L\tp\t+\tq\t+\t0M\n",
    "int_spellings": "S\ta\t+7\t*\nS\tb\t007\t*\nS\tc\t1_0\t*\nS\td\t 5 \t*\n"
                     "E\te\ta+\t 1\t2 \tb+\t0_0\t3\t*\nE\tf\tc-\t+2\t1_0\td+\t0\t5\t*\n",
    "zero_length": "S\tz\t0\t*\nS\ty\t3\t*\nE\te\tz+\t0\t0\ty+\t0\t3\t*\nL\tz\t+\ty\t+\t0M\n",
    "empty": "",
    "only_segments": "S\t1\t4\t*\nS\t2\t*\nS\t3\t9\t*\n",
    "unknown_then_split_warn": "H\tVN:Z:2.0\n#comment\nS\ta\t4\t*\nL\ta\t+\tq\t-\t0M\nW\tx\n",
    "malformed_l": "S\ta\t4\t*\nE\te\ta+\t0\t2\tzz+\t0\t1\t*\nL\ta\t+\n",
    "gfa2ish_links": "S\tu\t3\t*\nS\tv\t3\t*\nL\tu+\tv-\t0M\tRC:i:5\nL\tu\tv\t*\n",
    "crlf": "S\ta\t4\t*\r\nS\tb\t4\t*\r\nE\te\ta+\t0\t2\tb-\t2\t4\t*\r\nL\ta\t+\tb\t-\t0M\r\n",
    "weights_float": "S\ta\t6\t*\nS\tb\t6\t*\nE\te\ta+\t0\t3\tb+\t3\t6\t*\tRC:f:2.5\n"
                     "E\tf\ta+\t0\t3\tb+\t3\t6\t*\tRC:f:-1.5\nL\ta\t+\tb\t+\t0M\tRC:i:300\n",
    "p_and_o": "S\ta\t6\t*\nS\tb\t6\t*\nP\tp1\ta+,b-\t*\nO\to1\ta+ b-\nE\te\ta+\t1\t2\tb+\t1\t2\t*\n",
    "short_p": "S\ta\t6\t*\nP\tp1\n",
}


def run(path: Path, mode: dict) -> dict:
    sys.path.insert(0, REF)
    import numpy as np
    from gfa2network import parse_gfa

    rec: dict = {"warnings": [], "exc": None}
    with warnings.catch_warnings(record=True) as ws:
        warnings.simplefilter("always")
        try:
            A, nodes = parse_gfa(str(path), build_graph=False, build_matrix=True, return_node_list=True,
                                 split_on_alignment=True, **mode)
        except Exception as e:  # noqa: BLE001 - recorded as data
            rec["exc"] = [type(e).__name__, str(e)]
            A = nodes = None
        rec["warnings"] = [[w.category.__name__, str(w.message)] for w in ws]
    if A is not None:
        arrs = {"indptr": A.indptr, "indices": A.indices} if A.format == "csr" else {"row": A.row, "col": A.col}
        arrs["data"] = A.data
        rec.update(format=A.format, shape=list(A.shape), dtype=str(A.dtype),
                   arrays={k: [str(v.dtype), base64.b64encode(np.ascontiguousarray(v).tobytes()).decode()]
                           for k, v in arrs.items()},
                   nodes=[base64.b64encode(x if isinstance(x, bytes) else x.encode()).decode() for x in nodes],
                   nodes_bytes=bool(nodes) and isinstance(nodes[0], bytes))
    return rec


def main() -> None:
    INPUTS.mkdir(exist_ok=True)
    for name, text in SPLIT.items():
        (INPUTS / f"{name}.gfa").write_bytes(text.encode("latin-1"))
    files = sorted(INPUTS.glob("*.gfa")) + sorted((HERE / "inputs").glob("*"))
    out = {}
    for f in files:
        for mname, mode in MODES.items():
            if (f.stat().st_size > 100_000 or f.name.startswith("syn3k")) and mname != "default":
                continue  # the large fixtures in one mode keep split.json small
            out[f"{f.parent.name}/{f.name}|{mname}"] = run(f, mode)
    dst = HERE / "expected" / "split.json"
    dst.write_text(json.dumps({"modes": MODES, "cases": out}, indent=0, sort_keys=True))
    print(f"{len(out)} cases -> {dst}")


if __name__ == "__main__":
    main()
