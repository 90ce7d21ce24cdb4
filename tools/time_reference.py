#!/usr/bin/env python3
"""Time the REAL reference (sclipman/gfa2network) on this repo's synthetic generator.

Container-only (imports /root/reference; the reference never travels to the GPU box).
SURVEY.md §8(d): when the build's generator bytes differ from the survey's probe files,
re-time the reference on the build's own files before quoting speed-ups.  Times
`parse_gfa(path, build_graph=False, build_matrix=True, return_node_list=True, **mode)`
followed by `convert_format(A, "csr")`, single process (GIL: 1 core), warm page cache.

usage: python tools/time_reference.py C2 [C3 C4 ...]   -> profiles/r02/reference_cpu_times.json
       C4 is timed on the gzip file (64 MiB-uncompressed members, level 6: SURVEY.md §8(d)),
       the same bytes bench.py's end_to_end leg converts.
"""
import gzip
import json
import resource
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
OUT = ROOT / "profiles" / "r02" / "reference_cpu_times.json"


def main(names):
    sys.path.insert(0, "/root/reference")
    from gfa2network import convert_format, parse_gfa  # the reference (container only)

    from gfa2network_amd import synth

    results = json.loads(OUT.read_text()) if OUT.exists() else {}
    for name in names:
        wl = synth.WORKLOADS[name]
        data = synth.host_bytes(wl.n_segments, wl.n_links, seed=0, rc_tag=wl.rc_tag)
        gz = name == "C4"
        path = Path(f"/tmp/g2n_{name}.gfa" + (".gz" if gz else ""))
        if gz:
            from bench import write_gz_members

            write_gz_members(data, str(path), threads=8)
        else:
            path.write_bytes(data)
        mode = dict(wl.mode)
        t0 = time.perf_counter()
        A, nodes = parse_gfa(str(path), build_graph=False, build_matrix=True, return_node_list=True, **mode)
        t1 = time.perf_counter()
        C = convert_format(A, "csr")
        t2 = time.perf_counter()
        results[name] = {
            "workload": wl.note, "mode": mode or "default", "input_bytes": len(data),
            "file": path.name, "file_bytes": path.stat().st_size, "n_links": wl.n_links,
            "parse_gfa_s": round(t1 - t0, 3), "convert_csr_s": round(t2 - t1, 3), "total_s": round(t2 - t0, 3),
            "M_edges_per_s": round(wl.n_links / (t2 - t0) / 1e6, 4), "n": int(C.shape[0]), "nnz": int(C.nnz),
            "peak_rss_gb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 2),
            "host": "build container, Intel Xeon 8 vCPU, 1 core busy (GIL)",
        }
        print(name, results[name], flush=True)
        OUT.parent.mkdir(parents=True, exist_ok=True)
        OUT.write_text(json.dumps(results, indent=1))
        del A, nodes, C, data
        path.unlink()


if __name__ == "__main__":
    main(sys.argv[1:] or ["C2"])
