#!/usr/bin/env python3
"""Golden fixtures for ``gfa2network export --format edge-list`` from the REAL reference.

Runs ONLY in the build container, where the pure-Python reference is importable from
/root/reference.  For every input under tests/golden/inputs and both ``--bidirected``
settings it calls the reference's ``cli.main(["export", IN, "--format", "edge-list",
(--bidirected), "--output", OUT])`` (cli.py:264-281) in-process and records:
  * the bytes written to OUT (also on failure: the loop streams, so a failing record
    leaves the lines before it),
  * the exception type + message (or null),
  * the RuntimeWarnings emitted (parser.py:117-131).
Output: tests/golden/expected/export.json (plain data; nothing here is imported by the
product, the GPU tests or bench.py).
"""
from __future__ import annotations

import base64
import json
import sys
import tempfile
import warnings
from pathlib import Path

REF = "/root/reference"
HERE = Path(__file__).resolve().parent
INPUTS = HERE / "inputs"


def main() -> None:
    sys.path.insert(0, REF)
    from gfa2network import cli  # noqa: E402  (the reference)

    out = {}
    with tempfile.TemporaryDirectory() as td:
        for inp in sorted(INPUTS.iterdir()):
            for bidir in (False, True):
                dest = Path(td) / "edges.tsv"
                if dest.exists():
                    dest.unlink()
                argv = ["export", str(inp), "--format", "edge-list", "--output", str(dest)]
                if bidir:
                    argv.insert(4, "--bidirected")
                exc = None
                with warnings.catch_warnings(record=True) as w:
                    warnings.simplefilter("always")
                    try:
                        cli.main(argv)
                    except Exception as e:  # noqa: BLE001 - recorded as data
                        exc = [type(e).__name__, str(e)]
                text = dest.read_bytes() if dest.exists() else None
                out[f"{inp.name}|{int(bidir)}"] = {
                    "text_b64": None if text is None else base64.b64encode(text).decode(),
                    "exc": exc,
                    "warnings": [str(x.message) for x in w if issubclass(x.category, RuntimeWarning)],
                }
    (HERE / "expected" / "export.json").write_text(json.dumps(out, indent=0, sort_keys=True))
    print(f"{len(out)} export cases")


if __name__ == "__main__":
    main()
