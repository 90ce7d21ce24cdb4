#!/usr/bin/env python3
"""Benchmark of the MI355X GFA -> CSR path (BASELINE.json metric).

One "step" = one full pass of the hot path over one HBM-resident synthetic GFA: raw bytes
already in HBM -> CSR (indptr / indices / data) in HBM, i.e. g2n_build_device() — lines,
classify, parse + weights, first-touch node ids, node-name blob, triplets and (default mode)
the A.maximum(A.T) symmetrisation.  The gzip inflate and the PCIe copy are host ingest,
measured separately (the end_to_end leg).

* `--gpus 1` (default): C4 of BASELINE.json (50M S / 200M L, default flags), the north star's
  200M-edge config, is `value`.  The same line carries `scaling_reference`: C5 (the multi-GPU
  config) built by one GPU alone and through the sharded protocol at one rank, with decimal and
  hashed segment names — the first point of the N-GPU curve on the N-GPU workload.
* `--gpus N > 1`: C5 as ONE file byte-range-sharded over N ranks (strong scaling: the total work
  is fixed), one process per GPU over RCCL.  Under `torch.distributed.run` the ranks come from its
  environment; started plainly (`python bench.py --gpus N`, no WORLD_SIZE) the script launches the
  N rank processes itself before anything touches a GPU.  Every rank checks that the process group
  holds exactly N ranks on the nccl backend and exits non-zero otherwise.  `value` = the file's
  edge records / max-over-ranks time (decimal names: the fast path); `alt_paths.hashed_names` times
  the general owner protocol on the same dimensions with hashed names.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.29 TB/s measured copy)


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default=None, choices=["C2", "C3", "C4", "C5"],
                    help="default: C4 on one GPU (the headline config), C5 byte-range-sharded over N > 1 ranks")
    ap.add_argument("--scale", type=float, default=1.0, help="shrink the workload (debug only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-links", type=int, default=12_000_000)
    ap.add_argument("--phases", action="store_true", help="print per-phase ms to stderr")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the end-to-end leg (file on the page cache -> scipy CSR + node list in host memory)")
    ap.add_argument("--e2e-only", action="store_true", help="only the end-to-end leg")
    ap.add_argument("--no-alt", action="store_true", help="skip the hash-dictionary comparison build")
    ap.add_argument("--names", default="decimal", choices=["decimal", "hashed", "permuted", "prefixed"],
                    help="segment names of the synthetic file: decimal ids 1..N (the configs' layout), hashed "
                         "(unique non-decimal names: the hash dictionary / the general sharded protocol) or permuted "
                         "(decimal names out of S order: the direct-address dictionary)")
    ap.add_argument("--force-protocol", action="store_true",
                    help="sharded runs: the general owner protocol even where the decimal fast path (or, on one "
                         "rank, no exchange at all) applies — to time the protocol itself")
    ap.add_argument("--no-c5-reference", action="store_true",
                    help="--gpus 1: skip the C5 legs (one GPU alone and sharded at one rank) the N-GPU curve starts from")
    ap.add_argument("--shard", action="store_true",
                    help="byte-range-shard the workload's one file over the ranks (gfa2network_amd/shard.py; "
                         "always on for C5)")
    return ap.parse_args()


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def needs_launch(n_gpus: int, env=None) -> bool:
    """`python bench.py --gpus N > 1` started without a launcher (no WORLD_SIZE in the environment)
    starts its own N ranks."""
    env = os.environ if env is None else env
    return n_gpus > 1 and "WORLD_SIZE" not in env


def launch_ranks(n: int, argv: list, script: str | None = None, env=None, poll_s: float = 0.2) -> int:
    """One child process per rank (RANK = LOCAL_RANK = r, WORLD_SIZE = n, MASTER_ADDR 127.0.0.1, a
    free MASTER_PORT), each running `script` (this file) with `argv`; the parent never touches a GPU
    (no HIP call happens before the children exist, and nothing is exec'ed).  Waits for all of them;
    the first child that fails has the others terminated.  Returns the job's exit code (0, or the
    first failure's, negative signals mapped to 128 + signal)."""
    import subprocess

    base = dict(os.environ if env is None else env)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n))
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, script or str(Path(__file__).resolve())] + list(argv), env=e))
    rc, pending = 0, list(procs)
    while pending:
        for p in list(pending):
            c = p.poll()
            if c is None:
                continue
            pending.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                for q in pending:
                    q.terminate()
        if pending:
            time.sleep(poll_s)
    return rc


def check_world(n_gpus: int, world: int, backend: str) -> None:
    """The process group must be exactly the N ranks `--gpus N` asked for, over RCCL (nccl)."""
    if world != n_gpus:
        raise SystemExit(f"bench.py: --gpus {n_gpus} but the process group holds {world} rank(s); "
                         f"run `python bench.py --gpus {n_gpus}` (it launches its ranks) or torch.distributed.run "
                         f"with --nproc-per-node {n_gpus}")
    if backend != "nccl":
        raise SystemExit(f"bench.py: process group backend is {backend!r}, not nccl (RCCL)")


def _dist_setup(n_gpus: int, always: bool = False):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or always:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(_free_port())
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        import torch
        import torch.distributed as dist

        from datetime import timedelta

        torch.cuda.set_device(local)
        # a collective that never completes ends the run (exit non-zero) instead of holding the node
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local), timeout=timedelta(minutes=5))
        check_world(n_gpus, dist.get_world_size(), dist.get_backend())
        world = dist.get_world_size()
    elif n_gpus != world:
        check_world(n_gpus, world, "nccl")
    return world, rank, local


def _barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def _max_over_ranks(world, value: float) -> float:
    if world == 1:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def algorithmic_bytes(input_bytes: int, n_nodes: int, nnz: int, w_dtype: int, w_idx: int = 4) -> int:
    """B_alg = B_in + (n+1) w_idx + nnz (w_idx + w_dtype)."""
    return input_bytes + (n_nodes + 1) * w_idx + nnz * (w_idx + w_dtype)


def config_leg(lib, nat, synth, wl, device: int, steps: int, warmup: int) -> dict:
    """One more BASELINE config on this GPU, device-resident like the headline (C2 / C3 beside C4):
    ms per build (host clock around g2n_build_device, which returns after its stream drained),
    edge records/s, phase times (hipEvents) and the whole-path fraction of HBM peak."""
    dev_in = synth.DeviceInput(wl.n_segments, wl.n_links, seed=0, rc_tag=wl.rc_tag, device=device)
    ctx = lib.g2n_context_create(device)
    mode = dict(wl.mode)
    o = nat.make_options(dtype="float64", output=nat.OUT_CSR, want_node_names=True, device=device,
                         directed=mode.get("directed", True), bidirected=mode.get("bidirected", False),
                         weight_tag=mode.get("weight_tag"))
    res = nat.Result()
    phases = []
    try:
        for k in range(warmup + steps):
            if k == warmup:
                t0 = time.perf_counter()
            rc = lib.g2n_build_device(ctx, dev_in.ptr, dev_in.len, ctypes.byref(o), ctypes.byref(res))
            if rc != 0:
                raise RuntimeError(f"{wl.name}: {nat.status_name(rc)}: {nat.last_error()}")
            if k >= warmup:
                ph = {}
                for j in range(res.n_phases):
                    name = res.phase_names[j].decode()
                    if not name.startswith("_"):
                        ph[name] = ph.get(name, 0.0) + res.phase_ms[j]
                phases.append(ph)
        dt = (time.perf_counter() - t0) / steps
    finally:
        lib.g2n_context_destroy(ctx)
        dev_in.free()
    avg = {k: sum(p.get(k, 0.0) for p in phases) / len(phases) for k in phases[0]}
    dev_ms = sum(avg.values())
    b_alg = algorithmic_bytes(int(res.input_bytes), int(res.n_nodes), int(res.nnz), 8)
    traffic, src = build_traffic(wl.name)
    return {"workload": f"{wl.name}: {wl.note}", "ms_per_step": round(dt * 1e3, 3),
            "m_edges_per_s": round(int(res.n_edges) / dt / 1e6, 2),
            "gb_per_s_ingested": round(int(res.input_bytes) / dt / 1e9, 2), "nnz": int(res.nnz),
            "device_ms_per_step": round(dev_ms, 3), "phase_ms": {k: round(v, 3) for k, v in avg.items()},
            "pipeline_roofline": {"bound": "hbm", "b_alg_bytes": b_alg,
                                  "frac": round(b_alg / (dev_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                  "traffic": traffic, "traffic_source": src}}


def cpu_baseline(workload, links: int) -> dict:
    """The oracle (C++ restatement of the reference, 1 thread) on a bounded sample of the
    same generator: segments scaled with the links so the S:L ratio is kept."""
    from gfa2network_amd import synth
    from oracle import oracle

    oracle.build()
    segs = max(1, int(workload.n_segments * links / workload.n_links))
    data = synth.host_bytes(segs, links, seed=0, rc_tag=workload.rc_tag)
    mode = dict(workload.mode)
    t0 = time.perf_counter()
    o = oracle.run(data, **mode)
    dt = time.perf_counter() - t0
    assert o.status == 0
    return {"value": round(links / dt / 1e6, 4), "unit": "M edges/s", "cores": 1, "kind": "port",
            "sample": f"{segs} S / {links} L lines of the {workload.name} generator ({len(data) / 1e9:.2f} GB), "
                      f"oracle/g2n_oracle.cpp single thread, {dt:.1f} s"}


def write_gz_members(data, path: str, member_bytes: int = 64 << 20, level: int = 6, threads: int = 16) -> int:
    """Multi-member gzip (64 MiB-uncompressed members, level 6), members
    deflated in parallel (zlib releases the GIL).  Returns the compressed size."""
    import struct
    import zlib
    from concurrent.futures import ThreadPoolExecutor

    mv = memoryview(data)

    def one(off):
        chunk = mv[off:off + member_bytes]
        co = zlib.compressobj(level, zlib.DEFLATED, -zlib.MAX_WBITS)
        body = co.compress(chunk) + co.flush()
        return (b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\xff" + body
                + struct.pack("<II", zlib.crc32(chunk), len(chunk) & 0xFFFFFFFF))

    total = 0
    with open(path, "wb") as fh, ThreadPoolExecutor(threads) as ex:
        for m in ex.map(one, range(0, len(data), member_bytes)):
            fh.write(m)
            total += len(m)
    return total


def write_gz_single(data, path: str, level: int = 6, threads: int = 16, piece: int = 32 << 20) -> int:
    """ONE gzip member over the whole input (pigz's layout: pieces deflated in parallel, each primed
    with the 32 KiB before it and ended by a sync flush, so back-references cross the piece
    boundaries; gzip.open reads it as one deflate stream).  Returns the compressed size."""
    import struct
    import zlib
    from concurrent.futures import ThreadPoolExecutor

    mv = memoryview(data)
    offs = list(range(0, len(data), piece)) or [0]

    def one(off):
        last = off + piece >= len(data)
        co = zlib.compressobj(level, zlib.DEFLATED, -zlib.MAX_WBITS,
                              **({"zdict": bytes(mv[max(0, off - 32768):off])} if off else {}))
        chunk = mv[off:off + piece]
        return co.compress(chunk) + co.flush(zlib.Z_FINISH if last else zlib.Z_SYNC_FLUSH), zlib.crc32(chunk), len(chunk)

    total, crc = 10, 0
    with open(path, "wb") as fh, ThreadPoolExecutor(threads) as ex:
        fh.write(b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\xff")
        for body, c, n in ex.map(one, offs):
            fh.write(body)
            total += len(body)
            crc = _crc32_combine(crc, c, n)
        fh.write(struct.pack("<II", crc, len(data) & 0xFFFFFFFF))
    return total + 8


def _crc32_combine(crc1: int, crc2: int, len2: int) -> int:
    """zlib's crc32_combine (CRC of A+B from CRC(A), CRC(B), len(B)) by GF(2) matrix powers."""
    def times(mat, vec):
        s, i = 0, 0
        while vec:
            if vec & 1:
                s ^= mat[i]
            vec >>= 1
            i += 1
        return s

    def square(mat):
        return [times(mat, mat[n]) for n in range(32)]

    if len2 <= 0:
        return crc1
    odd = [0xEDB88320] + [1 << n for n in range(31)]
    even = square(odd)
    odd = square(even)
    while True:
        even = square(odd)
        if len2 & 1:
            crc1 = times(even, crc1)
        len2 >>= 1
        if not len2:
            break
        odd = square(even)
        if len2 & 1:
            crc1 = times(odd, crc1)
        len2 >>= 1
        if not len2:
            break
    return crc1 ^ crc2


def write_bgzf(data, path: str, level: int = 6, threads: int = 16) -> int:
    """BGZF (htslib's bgzip layout: members of 65280 input bytes, 'BC' size subfield, EOF marker),
    members deflated in parallel batches.  Returns the compressed size."""
    import struct
    import zlib
    from concurrent.futures import ThreadPoolExecutor

    mv, blk, per = memoryview(data), 65280, 512

    def batch(off):
        out = bytearray()
        for o in range(off, min(off + blk * per, len(data)), blk):
            chunk = mv[o:o + blk]
            co = zlib.compressobj(level, zlib.DEFLATED, -zlib.MAX_WBITS)
            body = co.compress(chunk) + co.flush()
            out += (b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00"
                    + struct.pack("<H", 12 + 6 + len(body) + 8 - 1) + body
                    + struct.pack("<II", zlib.crc32(chunk), len(chunk)))
        return bytes(out)

    total = 0
    with open(path, "wb") as fh, ThreadPoolExecutor(threads) as ex:
        for m in ex.map(batch, range(0, len(data), blk * per)):
            fh.write(m)
            total += len(m)
        eof = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
        fh.write(eof)
    return total + len(eof)


def end_to_end(wl, n_s: int, n_l: int, device: int) -> dict:
    """a GFA file on the warm page cache -> parse_gfa(..., return_node_list=True)
    + convert_format(A, "csr") in host memory, through the product's path (g2n_build_from_path:
    parallel member inflate, pinned staged H2D, GPU pipeline, D2H, scipy/list objects).  Plain
    and multi-member gzip inputs; one warm-up, then one timed run each."""
    import shutil
    import tempfile

    import numpy as np

    from gfa2network_amd import _native as nat
    from gfa2network_amd import synth
    from gfa2network_amd.api import convert_format, finalize

    threads = int(os.environ.get("G2N_HOST_THREADS", "0")) or min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    data = synth.host_bytes(n_s, n_l, seed=0, rc_tag=wl.rc_tag, threads=threads)
    tmp = tempfile.mkdtemp(prefix="g2n_e2e_", dir=os.environ.get("TMPDIR") or "/tmp")
    out = {"host_threads": threads, "input_bytes": len(data)}
    try:
        plain = os.path.join(tmp, "c.gfa")
        with open(plain, "wb") as fh:
            fh.write(data)
        gz = os.path.join(tmp, "c.gfa.gz")
        out["gz_bytes"] = write_gz_members(data, gz, threads=threads)
        gz1 = os.path.join(tmp, "c.single.gfa.gz")
        out["gz_single_bytes"] = write_gz_single(data, gz1, threads=threads)
        bgz = os.path.join(tmp, "c.bgzf.gz")
        out["bgzf_bytes"] = write_bgzf(data, bgz, threads=threads)
        out["prep_s"] = round(time.perf_counter() - t0, 1)
        del data
        mode = dict(wl.mode)
        dt = np.dtype("float64")
        opts = nat.make_options(dtype="float64", output=nat.OUT_PARSE, want_node_names=True, device=device,
                                directed=mode.get("directed", True), bidirected=mode.get("bidirected", False),
                                weight_tag=mode.get("weight_tag"))
        for name, path in (("plain", plain), ("gzip_64MiB_members", gz), ("gzip_single_member", gz1),
                           ("bgzf_gpu_inflate", bgz)):
            for it in range(2):
                t0 = time.perf_counter()
                raw = nat.build_from_path(path, opts)
                t1 = time.perf_counter()
                A, nodes = finalize(raw, dtype=dt, return_node_list=True, raw_bytes_id=False, verbose=False)
                C = convert_format(A, "csr")
                t2 = time.perf_counter()
            assert C.format == "csr" and len(nodes) == raw.n_nodes
            dev_ms = sum(v for k, v in raw.phase_ms.items() if not k.startswith("_"))
            wall = t2 - t0
            ok = _digest_ok(wl.name, n_s, n_l, C, nodes)  # after the timed region
            out[name] = {
                "wall_s": round(wall, 3), "m_edges_per_s": round(raw.n_edges / wall / 1e6, 2),
                "gb_per_s_ingested": round(raw.input_bytes / wall / 1e9, 2),
                "stages_ms": {"read_inflate": round(raw.host_ms["read"], 1), "staged_h2d": round(raw.host_ms["h2d"], 1),
                              "device": round(dev_ms, 1), "d2h": round(raw.host_ms["d2h"], 1),
                              "native_total": round((t1 - t0) * 1e3, 1),
                              "gpu_inflate": round(raw.phase_ms.get("gz_inflate", 0.0), 1),
                              "python_objects": round((t2 - t1) * 1e3, 1)},
                "nnz": int(C.nnz), "n_nodes": len(nodes), "digest_ok": ok}
            del A, C, nodes, raw
        # the convert CLI end to end (cli.py:193-250): gzip file -> .npz + .nodes.tsv on disk
        from gfa2network_amd.cli import main as cli_main

        npz = os.path.join(tmp, "c.npz")
        argv = ["convert", gz, "--matrix", npz] + (["--undirected"] if not mode.get("directed", True) else []) + \
            (["--bidirected"] if mode.get("bidirected") else []) + \
            (["--weight-tag", mode["weight_tag"]] if mode.get("weight_tag") else [])
        import contextlib
        import io

        with contextlib.redirect_stdout(io.StringIO()):
            t0 = time.perf_counter()
            cli_main(argv)
            wall = time.perf_counter() - t0
        out["cli_convert_gzip"] = {
            "argv": "convert c.gfa.gz --matrix c.npz" + ("".join(" " + a for a in argv[4:])),
            "wall_s": round(wall, 3), "m_edges_per_s": round(n_l / wall / 1e6, 2),
            "npz_bytes": os.path.getsize(npz), "nodes_tsv_bytes": os.path.getsize(npz + ".nodes.tsv"),
            "writers": "native (g2n_write_npz / g2n_write_node_map, host threads)"}
        import scipy.sparse as sp

        with open(npz + ".nodes.tsv", "rb") as fh:  # utils.py:108-114: "<index>\t<name>\n" per node
            names = [ln.split(b"\t", 1)[1].decode() for ln in fh.read().splitlines()]
        out["cli_convert_gzip"]["digest_ok"] = _digest_ok(wl.name, n_s, n_l, sp.load_npz(npz).tocsr(), names)
        del names
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    ref = {"C4": 1295.5}.get(wl.name)  # reference parse_gfa+convert_format, gzip C4, 1 core
    if ref:
        out["reference_cpu_s"] = ref
        out["speedup_vs_reference_gzip"] = round(ref / out["gzip_64MiB_members"]["wall_s"], 1)
    # the reference re-timed on THIS generator's gzip bytes (tools/time_reference.py, build container)
    rt = ROOT / "profiles" / "r02" / "reference_cpu_times.json"
    if rt.exists():
        same = json.loads(rt.read_text()).get(wl.name)
        if same and same.get("file_bytes") == out.get("gz_bytes"):
            out["reference_same_file"] = {
                "total_s": same["total_s"], "file_bytes": same["file_bytes"], "host": same.get("host"),
                "speedup": round(same["total_s"] / out["gzip_64MiB_members"]["wall_s"], 1),
                "note": "identical .gz bytes (64 MiB members); timed on the 8-vCPU build container"}
    return out


def _digest_ok(workload: str, n_s: int, n_l: int, C, nodes):
    """The end-to-end result against the oracle's digest of the same generator bytes
    (tests/golden/expected/synth_digests.json, tests/golden/make_synth_digests.py): sha256 of the
    int32 indptr | indices | data of the CSR parse_gfa + convert_format return, and of the names in
    id order.  None when the workload has no digest (scaled runs)."""
    import hashlib

    import numpy as np

    doc = json.loads((ROOT / "tests" / "golden" / "expected" / "synth_digests.json").read_text()).get(workload)
    if not doc or (doc["n_segments"], doc["n_links"]) != (n_s, n_l):
        return None
    want = doc["parse"] if doc["parse"]["format"] == "csr" else doc["csr"]  # what convert_format(A, "csr") gives
    h = hashlib.sha256()
    for a in (C.indptr.astype(np.int32, copy=False), C.indices.astype(np.int32, copy=False), C.data):
        h.update(np.ascontiguousarray(a).tobytes())
    names = hashlib.sha256("".join(nodes).encode()).hexdigest()
    return h.hexdigest() == want["digest"] and names == doc["names"]


def _line_start_device(ptr: int, length: int, nominal: int) -> int:
    """The first line start at or after `nominal` in a device-resident file (shard.line_ranges's
    rule), from small windows copied to the host."""
    import numpy as np

    from gfa2network_amd import synth

    if nominal <= 0 or nominal >= length:
        return min(max(nominal, 0), length)
    pos = nominal - 1
    while pos < length:
        n = min(1 << 16, length - pos)
        win = np.empty(n, dtype=np.uint8)
        synth._lib().g2n_synth_download(win.ctypes.data, ptr + pos, n)
        k = np.flatnonzero(win == 0x0A)
        if len(k):
            return pos + int(k[0]) + 1
        pos += n
    return length


def sharded_leg(args, wl, world: int, rank: int, local: int, names: str, force_protocol: bool = False,
                one_gpu: bool = True) -> dict:
    """ONE synthetic file byte-range-sharded over the group's ranks.  Every rank
    holds the whole file in its HBM (the generator is deterministic: the same bytes on every rank;
    generation is untimed) and builds only its line-aligned range through the sharded protocol
    (gfa2network_amd/shard.py: decimal names — one all-gather of the ranges' evidence, the range
    parsed straight into global ids; other names — the owner protocol: keys all-to-all to their
    owners, owner dedup, global ids by ranking; then triplets all-to-all to their row owners and
    the rank's CSR row slice).  Strong scaling: the total work is the one file.  one_gpu: rank 0
    first times the same file built by one GPU alone (g2n_build_device), the scaling reference."""
    import torch
    import torch.distributed as dist

    from gfa2network_amd import _native as nat
    from gfa2network_amd import synth
    from gfa2network_amd.shard import HipEngine, build_sharded

    n_s = max(1, int(wl.n_segments * args.scale))
    n_l = max(1, int(wl.n_links * args.scale))
    dev_in = synth.DeviceInput(n_s, n_l, seed=0, rc_tag=wl.rc_tag, device=local, names=names)
    starts = [_line_start_device(dev_in.ptr, dev_in.len, r * dev_in.len // world) for r in range(world)] + [dev_in.len]
    lo, hi = starts[rank], starts[rank + 1]
    mode = dict(wl.mode)
    # copy_out=False: each rank's CSR slice stays in its engine's HBM arena, as the one-GPU build's
    # result stays in its context (no device-to-device copy into torch tensors)
    kw = dict(directed=mode.get("directed", True), bidirected=mode.get("bidirected", False),
              weight_tag=mode.get("weight_tag"), dtype="float64", force_protocol=force_protocol, copy_out=False)
    one = None
    lib = nat.load()
    try:
        if one_gpu and rank == 0:  # the whole file on one GPU: the scaling reference
            ctx = lib.g2n_context_create(local)
            o = nat.make_options(dtype="float64", output=nat.OUT_CSR, want_node_names=True, device=local,
                                 directed=kw["directed"], bidirected=kw["bidirected"], weight_tag=kw["weight_tag"])
            res = nat.Result()
            try:
                for i in range(max(1, args.warmup) + args.steps):
                    if i == max(1, args.warmup):
                        t0 = time.perf_counter()
                    rc = lib.g2n_build_device(ctx, dev_in.ptr, dev_in.len, ctypes.byref(o), ctypes.byref(res))
                    if rc != 0:
                        raise RuntimeError(f"one-GPU {wl.name}: {nat.status_name(rc)}: {nat.last_error()}")
                dt = (time.perf_counter() - t0) / args.steps
                one = {"ms_per_step": round(dt * 1e3, 3), "value": round(n_l / dt / 1e6, 2), "nnz": int(res.nnz),
                       "n_nodes": int(res.n_nodes)}
            finally:
                lib.g2n_context_destroy(ctx)
        dist.barrier()
        eng = HipEngine(local)
        try:
            buf = _DevBytes(dev_in.ptr + lo, hi - lo)
            for _ in range(args.warmup):
                build_sharded(buf, engine=eng, **kw)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            tms = []
            for _ in range(args.steps):
                res = build_sharded(buf, engine=eng, **kw)
                tms.append(res.timings_ms)
            torch.cuda.synchronize()
            dist.barrier()
            elapsed = _max_over_ranks(world, time.perf_counter() - t0)
            slice_nnz = torch.tensor([int(res.indices.numel())], dtype=torch.int64, device="cuda")
            dist.all_reduce(slice_nnz)
        finally:
            eng.close()
    finally:
        dev_in.free()
    value = res.n_edges * args.steps / elapsed / 1e6
    leg = {"value": round(value, 2), "ms_per_step": round(elapsed / args.steps * 1e3, 3),
           "gb_per_s_ingested": round(dev_in.len * args.steps / elapsed / 1e9, 2),
           "n_segments": n_s, "n_links": n_l, "input_bytes": dev_in.len, "n_nodes": res.n_nodes,
           "nnz": int(slice_nnz.item()), "segment_names": names,
           "id_path": ("decimal-id fast path" if res.fast_path else
                       "general owner protocol" + (" (forced at one rank)" if force_protocol else "")),
           "host_ms_per_stage_rank0": {k: round(sum(t.get(k, 0.0) for t in tms) / len(tms), 2) for k in tms[0]}}
    if one is not None:
        leg["one_gpu"] = one
        leg["speedup_vs_one_gpu"] = round(value / one["value"], 3)
        leg["same_shape_as_one_gpu"] = one["nnz"] == leg["nnz"] and one["n_nodes"] == leg["n_nodes"]
    return leg


def main_sharded(args, wl):
    """`--gpus N > 1` (or `--shard`): the N-rank line (module docstring)."""
    import torch.distributed as dist

    world, rank, local = _dist_setup(args.gpus, always=True)
    leg = sharded_leg(args, wl, world, rank, local, args.names, args.force_protocol)
    alt = None
    if not args.no_alt and args.names == "decimal":
        try:
            alt = sharded_leg(args, wl, world, rank, local, "hashed")
        except Exception as exc:  # noqa: BLE001 - the headline (decimal) leg is already measured
            alt = {"error": f"{type(exc).__name__}: {exc}"}
    mode = dict(wl.mode)
    line = {
        "metric": "M edges/sec GFA->CSR (device-resident), + GB/s ingested",
        "value": leg["value"], "unit": "M edge records/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": leg["ms_per_step"], "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u8/int64 (float64 weights)",
        "data": "synthetic (deterministic generator, gfa2network_amd/csrc/synth.h), generated in HBM on every rank",
        "world_size": world, "backend": dist.get_backend(),
        "config": {"workload": f"{wl.name}: {wl.note}, one file byte-range-sharded over {world} rank(s)"
                               + (f" x{args.scale}" if args.scale != 1 else ""),
                   "n_segments": leg["n_segments"], "n_links": leg["n_links"], "input_bytes": leg["input_bytes"],
                   "n_nodes": leg["n_nodes"], "nnz": leg["nnz"], "mode": mode or "default",
                   "output": "csr row slice per rank",
                   "parallelism": f"shard x{world} (RCCL: all-gather of the ranges' evidence, all-to-all of "
                                  f"triplets to row owners; hashed names: keys to owners, all-gather of order keys)",
                   "segment_names": args.names, "id_path": leg["id_path"]},
        "gb_per_s_ingested": leg["gb_per_s_ingested"],
        "host_ms_per_stage_rank0": leg["host_ms_per_stage_rank0"],
    }
    if "one_gpu" in leg:
        line["one_gpu"] = leg["one_gpu"]
        line["speedup_vs_one_gpu"] = leg["speedup_vs_one_gpu"]
    if alt is not None:
        line["alt_paths"] = {"hashed_names": dict(alt, note="the same dimensions with hashed segment names "
                                                  "(not 1..N): the general owner protocol over RCCL")}
    if rank == 0:
        print(json.dumps(line))
    dist.destroy_process_group()


def scaling_reference(args) -> dict:
    """The first point of the N-GPU curve on the N-GPU workload (C5), for the `--gpus 1` line: C5
    built by one GPU alone and through the sharded protocol at one rank (a world-1 RCCL group),
    decimal names (the fast path) and hashed names (the owner protocol forced at one rank, so the
    exchange steps run as they do at N > 1)."""
    import torch.distributed as dist

    from gfa2network_amd import synth

    wl = synth.WORKLOADS["C5"]
    world, rank, local = _dist_setup(1, always=True)
    try:
        out = {"workload": f"{wl.name}: {wl.note}", "world_size": world, "backend": dist.get_backend(),
               "decimal": sharded_leg(args, wl, world, rank, local, "decimal"),
               "hashed": sharded_leg(args, wl, world, rank, local, "hashed", force_protocol=True)}
    finally:
        dist.destroy_process_group()
    return out


def main():
    args = _args()
    if needs_launch(args.gpus):  # before anything touches a GPU: this process only waits for its ranks
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.workload is None:
        args.workload = "C5" if max(world_env, args.gpus) > 1 else "C4"
    if (args.workload == "C5" or args.shard) and not args.e2e_only:
        from gfa2network_amd import synth

        main_sharded(args, synth.WORKLOADS[args.workload])
        return
    if args.e2e_only:
        from gfa2network_amd import synth

        wl = synth.WORKLOADS[args.workload]
        print(json.dumps(end_to_end(wl, max(1, int(wl.n_segments * args.scale)),
                                    max(1, int(wl.n_links * args.scale)), 0)))
        return
    world, rank, local = _dist_setup(args.gpus)
    from gfa2network_amd import _native as nat
    from gfa2network_amd import synth

    lib = nat.load()
    wl = synth.WORKLOADS[args.workload]
    n_s = max(1, int(wl.n_segments * args.scale))
    n_l = max(1, int(wl.n_links * args.scale))
    dev_in = synth.DeviceInput(n_s, n_l, seed=rank, rc_tag=wl.rc_tag, device=local, names=args.names)
    ctx = lib.g2n_context_create(local)
    if not ctx:
        raise RuntimeError(nat.last_error())
    mode = dict(wl.mode)
    opts = nat.make_options(dtype="float64", output=nat.OUT_CSR, want_node_names=True, device=local,
                            directed=mode.get("directed", True), bidirected=mode.get("bidirected", False),
                            weight_tag=mode.get("weight_tag"))
    res = nat.Result()

    def step(o=None):
        rc = lib.g2n_build_device(ctx, dev_in.ptr, dev_in.len, ctypes.byref(o or opts), ctypes.byref(res))
        if rc != 0:
            raise RuntimeError(f"{nat.status_name(rc)}: {nat.last_error()}")
        ph = {}
        for k in range(res.n_phases):  # "_"-phases are host gaps between measured kernels
            name = res.phase_names[k].decode()
            if not name.startswith("_"):
                ph[name] = ph.get(name, 0.0) + res.phase_ms[k]
        return ph

    for _ in range(args.warmup):
        step()
    _barrier(world)
    lib.g2n_context_stream(ctx)
    phases = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        phases.append(step())  # returns after the pipeline stream drained
    _barrier(world)
    elapsed = time.perf_counter() - t0
    elapsed = _max_over_ranks(world, elapsed)

    n_edges, n_nodes, nnz, in_bytes = int(res.n_edges), int(res.n_nodes), int(res.nnz), int(res.input_bytes)
    # the same build through the hash dictionary (what inputs without decimal segment ids take)
    t_h, hash_ph = None, None
    if not args.no_alt:
        hopts = nat.make_options(dtype="float64", output=nat.OUT_CSR, want_node_names=True, device=local,
                                 directed=mode.get("directed", True), bidirected=mode.get("bidirected", False),
                                 weight_tag=mode.get("weight_tag"), test_flags=nat.TEST_DICT_HASH)
        step(hopts)
        t_h = time.perf_counter()
        hash_ph = step(hopts)
        t_h = time.perf_counter() - t_h
    # decimal names out of S order (a permutation of 1..N), and minigraph's prefixed names "s1".."sN" in S
    # order: the direct-address dictionary tier (S lines claim direct[v], each edge name one 4-byte read)
    alt_names = {}
    name_legs = {
        "permuted_names": ("permuted", "same dimensions and flags, segment names a permutation of 1..N (synth "
                           "names='permuted'): the direct-address dictionary (S lines claim direct[v], each edge "
                           "name one 4-byte read)"),
        "prefixed_names": ("prefixed", "same dimensions and flags, segment names 's1'..'sN' in S order (synth "
                           "names='prefixed', minigraph's layout): the direct-address dictionary with a one-byte "
                           "prefix"),
    }
    for leg, (nm, note) in (name_legs.items() if not args.no_alt and args.names == "decimal" else ()):
        perm = synth.DeviceInput(n_s, n_l, seed=rank, rc_tag=wl.rc_tag, device=local, names=nm)
        try:
            pph = []
            for i in range(1 + max(2, min(args.steps, 5))):
                t_p = time.perf_counter()
                rc = lib.g2n_build_device(ctx, perm.ptr, perm.len, ctypes.byref(opts), ctypes.byref(res))
                t_p = time.perf_counter() - t_p
                if rc != 0:
                    raise RuntimeError(f"{nat.status_name(rc)}: {nat.last_error()}")
                if i:
                    pph.append(({res.phase_names[k].decode(): res.phase_ms[k] for k in range(res.n_phases)
                                 if not res.phase_names[k].decode().startswith("_")}, t_p))
            p_avg = {k: sum(p[0].get(k, 0.0) for p in pph) / len(pph) for k in pph[0][0]}
            p_ms = sum(p[1] for p in pph) / len(pph) * 1e3
            alt_names[leg] = {
                "ms_per_step": round(p_ms, 3), "m_edges_per_s": round(int(res.n_edges) / (p_ms / 1e3) / 1e6, 2),
                "device_ms_per_step": round(sum(p_avg.values()), 3), "input_bytes": perm.len, "nnz": int(res.nnz),
                "phase_ms": {k: round(v, 3) for k, v in p_avg.items()}, "note": note}
        finally:
            perm.free()
    # export --format edge-list on the same input (the text rendered in HBM)
    t_x, x_ph, x_bytes = None, None, 0
    if not args.no_alt:
        xopts = nat.make_options(output=nat.OUT_EDGE_LIST, device=local)
        step(xopts)
        t_x = time.perf_counter()
        x_ph = step(xopts)
        t_x = time.perf_counter() - t_x
        x_bytes = int(res.nnz)
        step()  # leaves res describing the CSR build again
    w_dtype = 8
    ms_step = elapsed / args.steps * 1e3
    edges_total = n_edges * args.steps * world
    value = edges_total / elapsed / 1e6
    gbs = in_bytes * args.steps * world / elapsed / 1e9
    # per-phase device time (hipEvents on the pipeline stream), averaged over the steps
    avg = {k: sum(p.get(k, 0.0) for p in phases) / len(phases) for k in phases[0]}
    dev_ms = sum(avg.values())
    b_alg = algorithmic_bytes(in_bytes, n_nodes, nnz, w_dtype)
    # roofline of the dominant single kernel: its algorithmic bytes per launch / its event time
    counts = dict(n_lines=int(res.n_lines), n_edges=n_edges, n_nodes=n_nodes, in_bytes=in_bytes,
                  names_bytes=int(res.names_bytes), bidir=bool(mode.get("bidirected")),
                  keep=bool(mode.get("keep_directed_bidir")), n_s=n_s, w_dtype=w_dtype,
                  directed_csr=bool(mode.get("keep_directed_bidir")) or (not mode.get("bidirected")
                                                                        and mode.get("directed", True)),
                  lean="values" in phases[0], weighted=bool(mode.get("weight_tag")))
    cand = {ph: avg[ph] for ph in KERNEL_OF_PHASE if ph in avg}
    dom = max(cand, key=cand.get)
    dom_bytes, unit_desc = kernel_bytes(dom, **counts)
    achieved = dom_bytes / (avg[dom] / 1e3) / 1e9
    kname = KERNEL_OF_PHASE[dom]
    if dom == "parse" and (counts["bidir"] or counts["weighted"]):  # the extended tile-local instance
        kname = "g2n::k_tile_lean<0, false, true>"
    # (the committed PMC summary is C4's: other workloads report no traffic)
    traffic, traffic_src = measured_traffic(kname) if wl.name == "C4" and args.scale == 1 else (None, None)
    line = {
        "metric": "M edges/sec GFA->CSR (device-resident), + GB/s ingested",
        "value": round(value, 2),
        "unit": "M edge records/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/int64 (float64 weights)",
        "data": "synthetic (deterministic generator, gfa2network_amd/csrc/synth.h), generated in HBM",
        "config": {"workload": f"{wl.name}: {wl.note}" + (f" x{args.scale}" if args.scale != 1 else ""),
                   "n_segments": n_s, "n_links": n_l, "input_bytes_per_gpu": in_bytes, "n_nodes": n_nodes,
                   "nnz": nnz, "mode": mode or "default", "output": "csr", "parallelism": f"replica x{world}"},
        "gb_per_s_ingested": round(gbs, 2),
        "device_ms_per_step": round(dev_ms, 3),
        "phase_ms": {k: round(v, 3) for k, v in avg.items()},
        "pipeline_roofline": {"bound": "hbm", "b_alg_bytes": b_alg,
                              "achieved_gbs": round(b_alg / (dev_ms / 1e3) / 1e9, 1),
                              "peak_gbs": HBM_PEAK_GBS,
                              "frac": round(b_alg / (dev_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)},
        "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src, "algorithmic_bytes_per_launch": dom_bytes,
                     "per_unit": unit_desc, "ms_per_launch": round(avg[dom], 3),
                     "timing": "hipEvents on the pipeline stream around the kernel, averaged over the timed steps"},
    }
    if t_h is not None:
        line["alt_paths"] = {"hash_dictionary": {
            "ms_per_step": round(t_h * 1e3, 3), "m_edges_per_s": round(n_edges / t_h / 1e6, 2),
            "phase_ms": {k: round(v, 3) for k, v in hash_ph.items()},
            "note": "options.test_flags = G2N_TEST_DICT_HASH: segment names resolved through the GPU hash table (inputs whose S lines "
                    "are not named 1..N in order)"}}
    for leg, rec in alt_names.items():
        line.setdefault("alt_paths", {})[leg] = rec
    if t_x is not None:
        xt = x_ph.get("edge_text", 0.0)
        line.setdefault("alt_paths", {})["export_edge_list"] = {
            "ms_per_step": round(t_x * 1e3, 3), "m_edges_per_s": round(n_edges / t_x / 1e6, 2),
            "text_bytes": x_bytes, "phase_ms": {k: round(v, 3) for k, v in x_ph.items()},
            "edge_text_gbs": round((x_bytes + 8 * n_edges) / (xt / 1e3) / 1e9, 1) if xt else None,
            "note": "export --format edge-list (cli.py:264-281): the same parse with a stream-order COO, "
                    "then per-edge lengths, a scan and the rendered u\\tv lines in HBM (device-resident; "
                    "edge_text_gbs = (text bytes + 8 B ids per edge) / edge_text phase)"}
    if not args.no_alt and world == 1:
        # the same dimensions with no id locality (an L line's second segment uniform over all
        # segments): every entry's two rows fall in different CSR buckets, so none travels as one
        # pair element through the partition (g2n_sym.hip) — the assembly's worst case
        far = synth.DeviceInput(n_s, n_l, seed=rank, rc_tag=wl.rc_tag, device=local, names=args.names,
                                far_links=True)
        try:
            far_ph = []
            for i in range(1 + max(2, min(args.steps, 5))):
                rc = lib.g2n_build_device(ctx, far.ptr, far.len, ctypes.byref(opts), ctypes.byref(res))
                if rc != 0:
                    raise RuntimeError(f"{nat.status_name(rc)}: {nat.last_error()}")
                if i:
                    far_ph.append({res.phase_names[k].decode(): res.phase_ms[k] for k in range(res.n_phases)
                                   if not res.phase_names[k].decode().startswith("_")})
            far_avg = {k: sum(p.get(k, 0.0) for p in far_ph) / len(far_ph) for k in far_ph[0]}
            line.setdefault("alt_paths", {})["far_links"] = {
                "device_ms_per_step": round(sum(far_avg.values()), 3),
                "m_edges_per_s": round(int(res.n_edges) / (sum(far_avg.values()) / 1e3) / 1e6, 2),
                "nnz": int(res.nnz), "phase_ms": {k: round(v, 3) for k, v in far_avg.items()},
                "note": "same dimensions and flags, L lines' second segment uniform over all segments (no id "
                        "locality: no pair elements in the CSR partition); device time from the phase events"}
        finally:
            far.free()
        step()  # leaves res describing the headline build again
    if dom in ("insert_claim", "insert_lookup"):
        tps = 2 if mode.get("bidirected") else 1
        tpe = 4 if (mode.get("bidirected") and not mode.get("keep_directed_bidir")) else 2
        probes = n_s * tps if dom == "insert_claim" else n_edges * tpe
        line["roofline"]["random_access"] = random_ceiling(probes, avg[dom])
    lib.g2n_context_destroy(ctx)
    dev_in.free()
    if world == 1 and not args.no_alt and args.workload == "C4" and args.scale == 1:
        line["other_configs"] = {w: config_leg(lib, nat, synth, synth.WORKLOADS[w], local, max(args.steps, 10),
                                               max(args.warmup, 2)) for w in ("C2", "C3")}
    if world == 1 and not args.no_c5_reference and args.workload == "C4" and args.scale == 1:
        line["scaling_reference"] = scaling_reference(args)
    line["world_size"], line["backend"] = world, ("nccl" if world > 1 else None)
    if nat.TEST_FLAGS:  # (G2N_TEST_FLAGS forced a non-default path: the line says so)
        line["test_flags"] = int(nat.TEST_FLAGS)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(wl, min(args.cpu_sample_links, n_l))
    if rank == 0 and world == 1 and not args.no_e2e:
        line["end_to_end"] = end_to_end(wl, n_s, n_l, local)
    if rank == 0:
        if args.phases:
            print(json.dumps(avg, indent=1), file=sys.stderr)
        print(json.dumps(line))
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


class _DevBytes:
    """A device input as the protocol's byte-range argument (data_ptr / numel)."""

    def __init__(self, ptr, n):
        self.ptr, self.n = ptr, n

    def data_ptr(self):
        return self.ptr

    def numel(self):
        return self.n


KERNEL_OF_PHASE = {  # phases that time exactly one kernel launch per build
    "tiles": "g2n::k_tile_count",
    "parse": "g2n::k_tile_lean<0, true, false>",  # the tile-local lean parse (decimal ids, no K1, group slots)
    "insert_claim": "g2n::k_tile_lean<1, false>",  # the lean S-first hash tier (claim / edge passes)
    "insert_lookup": "g2n::k_tile_lean<2, false>",
    "direct_claim": "g2n::k_tile_lean<3, false>",  # the direct-address tier
    "direct_lookup": "g2n::k_tile_lean<4, false>",
    "triplets": "g2n::k_triplets<double>",
}


def kernel_bytes(phase, *, n_lines, n_edges, n_nodes, in_bytes, names_bytes, bidir, keep, n_s, w_dtype,
                 directed_csr=True, lean=False, weighted=False):
    """Algorithmic bytes one launch must move (inputs read once, outputs written once) and the
    per-unit figure it is built from."""
    tps = 2 if bidir else 1
    tpe = 4 if (bidir and not keep) else 2
    n_t = n_s * tps + n_edges * tpe
    d_o = 12 if bidir else 0  # orientation descriptor (u64 off + u32 len) per touch
    avg_key = names_bytes / max(n_nodes, 1)
    k_trip = tpe if tpe == 4 else (1 if directed_csr else 2)
    if phase == "tiles":  # K1 reads every byte once; 48 B of counts per 32 KiB tile
        return in_bytes, "B_in (K1: every input byte read once)"
    if phase == "parse" and lean:  # decimal ids: the COO coordinates (+ weights) per edge; the lean parse
        # writes no line starts / kinds and no S touch descriptors (names by arithmetic, k_names_dec)
        per_e = 4 * k_trip * 2 + (8 if weighted else 0)
        return in_bytes + per_e * n_edges, f"B_in + {per_e} B/edge (lean decimal-id parse)"
    if phase == "parse":  # every input byte once; line start + kind per line; descriptors per touch / edge
        per_t, per_e = 13 + d_o, 12
        return (in_bytes + 9 * n_lines + per_t * n_t + per_e * n_edges,
                f"B_in + 9 B/line + {per_t} B/touch + {per_e} B/edge")
    if phase in ("insert_claim", "insert_lookup"):
        k = n_s * tps if phase == "insert_claim" else n_edges * tpe
        per = 1 + 12 + d_o + avg_key + 32 + 4  # state, descriptor, key bytes, 32-B entry, slot / node id
        return (int(n_t * 1 + k * (per - 1)), f"1 B/touch + {per - 1:.1f} B per processed touch ({k} touches)")
    if phase == "direct_lookup":  # the edge lines' bytes, two 4-byte id reads and the COO per edge
        per = 8 + 4 * k_trip * 2
        return in_bytes + per * n_edges, f"B_in + {per} B/edge (direct-address edge pass)"
    if phase == "direct_claim":  # the S lines' bytes, one 4-byte claim + the name's offset / length per S line
        return in_bytes + 16 * n_s, "B_in + 16 B/S line (direct-address claim pass)"
    if phase == "triplets":
        per = 4 + 8 + tpe * 4 + k_trip * (4 + 4 + w_dtype)  # tb, w, node id per touch, COO out
        return n_edges * per, f"{per} B/edge"
    return in_bytes, "B_in"


def random_ceiling(records: int, ms: float):
    """The dictionary probe is one random 32-B record read per touch: its ceiling is the
    MI355X's random-record rate, measured by tools/microbench/randread.hip on a 4 GiB table
    (profiles/r01/randread_ceiling.jsonl), not the streaming HBM peak."""
    p = ROOT / "profiles" / "r01" / "randread_ceiling.jsonl"
    try:
        rows = [json.loads(x) for x in p.read_text().splitlines() if x.strip()]
    except (OSError, ValueError):
        return None
    rate = next((r["Grec_per_s"] for r in rows if r.get("shape") == "random 32B records" and r["table_GB"] > 1), None)
    if not rate:
        return None
    floor_ms = records / (rate * 1e9) * 1e3
    return {"records": records, "ceiling_Grec_per_s": rate, "floor_ms": round(floor_ms, 3),
            "achieved_Grec_per_s": round(records / (ms / 1e3) / 1e9, 2), "frac": round(floor_ms / ms, 3),
            "source": "profiles/r01/randread_ceiling.jsonl"}


PMC_SUMMARY = ROOT / "profiles" / "r06" / "pmc_c4.json"


def measured_traffic(kernel: str):
    """HBM bytes per launch for `kernel` (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md's gfx950
    correction) from the committed rocprofv3 PMC summary of this bench's C4 workload, with the
    commit of the sources it was measured on (tools/counter_table.py writes both), or None."""
    try:
        doc = json.loads(PMC_SUMMARY.read_text())
    except (OSError, ValueError):
        return None, None
    k = doc.get("kernels", {}).get(kernel, {})
    return k.get("traffic_bytes_per_launch"), {"file": str(PMC_SUMMARY.relative_to(ROOT)), "commit": doc.get("commit")}


def build_traffic(workload: str):
    """HBM bytes of one whole build of `workload` (every kernel's 2 x FETCH_SIZE + WRITE_SIZE times its
    launches) from its committed PMC summary (profiles/r06/pmc_<workload>.json, one build:
    tools/gpu_counters.sh with --steps 1 --warmup 0), or (None, None)."""
    f = PMC_SUMMARY.parent / f"pmc_{workload.lower()}.json"
    try:
        doc = json.loads(f.read_text())
    except (OSError, ValueError):
        return None, None
    # (not the input generator's kernels: k_synth_len / k_synth_write and its 64-bit scan, which a CSR
    # build of these configs never launches)
    ks = [v for n, v in doc.get("kernels", {}).items()
          if "synth" not in n and n != "g2n::k_scan_excl<unsigned long, unsigned long>"]
    if not ks or any("launches" not in k or k.get("traffic_bytes_per_launch") is None for k in ks):
        return None, None
    return (int(sum(k["traffic_bytes_per_launch"] * k["launches"] for k in ks)),
            {"file": str(f.relative_to(ROOT)), "commit": doc.get("commit"), "per": "build"})


if __name__ == "__main__":
    main()
