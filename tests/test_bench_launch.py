"""bench.py's multi-GPU launch and world checks (CPU): `python bench.py --gpus N` without a launcher
starts its N ranks itself, and a process group that is not exactly N ranks over nccl is refused."""
import os
import sys
import time
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def test_needs_launch_only_without_a_launcher():
    assert bench.needs_launch(8, env={})
    assert bench.needs_launch(2, env={"PATH": "/bin"})
    assert not bench.needs_launch(1, env={})
    assert not bench.needs_launch(8, env={"WORLD_SIZE": "8"})  # torch.distributed.run set it
    assert not bench.needs_launch(8, env={"WORLD_SIZE": "1"})  # ... and the world check then refuses it


def _stub(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text("import os, sys, time\n" + body)
    return str(p)


def test_launch_ranks_starts_every_rank_with_its_environment(tmp_path):
    out = tmp_path / "out"
    out.mkdir()
    script = _stub(tmp_path, f"""
r = os.environ["RANK"]
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
open(os.path.join({str(out)!r}, r), "w").write(" ".join(os.environ[k] for k in keys) + " " + " ".join(sys.argv[1:]))
""")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "MASTER_PORT")}
    rc = bench.launch_ranks(4, ["--gpus", "4", "--steps", "3"], script=script, env=env, poll_s=0.01)
    assert rc == 0
    got = {p.name: p.read_text().split() for p in out.iterdir()}
    assert sorted(got) == ["0", "1", "2", "3"]
    ports = {v[5] for v in got.values()}
    assert len(ports) == 1 and int(ports.pop()) > 0  # one rendezvous for the job
    for r, v in got.items():
        assert v[:5] == [r, r, "4", "4", "127.0.0.1"]
        assert v[6:] == ["--gpus", "4", "--steps", "3"]


def test_launch_ranks_fails_fast_and_stops_the_others(tmp_path):
    script = _stub(tmp_path, """
if os.environ["RANK"] == "1":
    sys.exit(3)
time.sleep(60)
""")
    t0 = time.perf_counter()
    rc = bench.launch_ranks(3, [], script=script, poll_s=0.01)
    assert rc == 3
    assert time.perf_counter() - t0 < 30  # the sleeping ranks were terminated, not waited for


def test_launch_ranks_maps_signals_to_a_nonzero_code(tmp_path):
    script = _stub(tmp_path, "import signal\nos.kill(os.getpid(), signal.SIGTERM)\n")
    assert bench.launch_ranks(1, [], script=script, poll_s=0.01) == 128 + 15


def test_check_world_refuses_a_wrong_group():
    bench.check_world(8, 8, "nccl")
    bench.check_world(1, 1, "nccl")
    with pytest.raises(SystemExit, match="holds 1 rank"):
        bench.check_world(8, 1, "nccl")
    with pytest.raises(SystemExit, match="holds 8 rank"):
        bench.check_world(2, 8, "nccl")
    with pytest.raises(SystemExit, match="not nccl"):
        bench.check_world(2, 2, "gloo")


def test_dist_setup_without_a_group_refuses_more_gpus(monkeypatch):
    # a plain `bench.py --gpus 4` that somehow skipped the launcher must not report a 1-rank run as 4 GPUs
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit, match="--gpus 4"):
        bench._dist_setup(4)
    assert bench._dist_setup(1) == (1, 0, 0)


def test_build_traffic_sums_every_build_kernel_once_per_launch():
    """The C2 / C3 legs' whole-build HBM traffic (bench.build_traffic): every kernel's per-launch
    2 x FETCH_SIZE + WRITE_SIZE times its launches, the input generator's kernels left out — from the
    committed summaries, and None for a workload without one."""
    import json

    for w in ("C2", "C3"):
        t, src = bench.build_traffic(w)
        doc = json.loads((bench.ROOT / src["file"]).read_text())
        want = sum(k["traffic_bytes_per_launch"] * k["launches"] for n, k in doc["kernels"].items()
                   if "synth" not in n and n != "g2n::k_scan_excl<unsigned long, unsigned long>")
        assert t == want > 0 and src["commit"] == doc["commit"] and src["per"] == "build"
    assert bench.build_traffic("C9") == (None, None)
