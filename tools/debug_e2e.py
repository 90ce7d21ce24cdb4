"""Debug: host entry points on large synthetic inputs (status, failing line)."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gfa2network_amd import _native as nat  # noqa: E402
from gfa2network_amd import synth  # noqa: E402

for scale in [float(x) for x in sys.argv[1:]] or [0.01, 0.1]:
    n_s, n_l = int(50e6 * scale), int(200e6 * scale)
    data = synth.host_bytes(n_s, n_l, seed=0, threads=16)
    opts = nat.make_options(dtype="float64", output=nat.OUT_PARSE, want_node_names=True)
    for how in ("buffer", "path"):
        if how == "buffer":
            raw = nat.build_from_buffer(data, opts)
        else:
            with tempfile.NamedTemporaryFile(suffix=".gfa") as f:
                f.write(data)
                f.flush()
                raw = nat.build_from_path(f.name, opts)
        line = ""
        if raw.status:
            ls = data.split(b"\n", raw.err_line + 1)
            line = ls[raw.err_line][:80] if raw.err_line >= 0 and raw.err_line < len(ls) else b"?"
        print(scale, how, len(data), "status", raw.status, "err_line", raw.err_line, line, raw.host_ms, flush=True)
