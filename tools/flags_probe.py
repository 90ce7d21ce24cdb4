"""Per-phase device ms of the C4 build under test flags (options.reserved[1]): how much a forced
rare path costs.  Usage: python tools/flags_probe.py FLAGS [FLAGS ...]   (0 = the default path)
e.g. 2 = TEST_NO_BUCKETS (the unweighted CSR through the general row-sum path)."""
import ctypes
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from gfa2network_amd import _native as nat
    from gfa2network_amd import synth

    lib = nat.load()
    wl = synth.WORKLOADS["C4"]
    dev = synth.DeviceInput(wl.n_segments, wl.n_links, seed=0, device=0)
    ctx = lib.g2n_context_create(0)
    res = nat.Result()
    for flags in [int(x) for x in sys.argv[1:]] or [0]:
        o = nat.make_options(dtype="float64", output=nat.OUT_CSR, want_node_names=True, device=0,
                             test_flags=flags)
        acc = {}
        for it in range(4):
            rc = lib.g2n_build_device(ctx, dev.ptr, dev.len, ctypes.byref(o), ctypes.byref(res))
            assert rc == 0, (rc, nat.last_error())
            if it:
                for k in range(res.n_phases):
                    name = res.phase_names[k].decode()
                    if not name.startswith("_"):
                        acc[name] = acc.get(name, 0.0) + res.phase_ms[k] / 3
        print(json.dumps({"flags": flags, "nnz": int(res.nnz), "phase_ms": {k: round(v, 3) for k, v in acc.items()},
                          "total_ms": round(sum(acc.values()), 3)}))
    lib.g2n_context_destroy(ctx)
    dev.free()


if __name__ == "__main__":
    main()
