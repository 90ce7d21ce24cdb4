#!/bin/bash
# SUM-CSR twin pairs: the synthetic / shard / diff GPU tests, C2 and the sharded C5 line; then the lean
# hash table's load factor A/B (tools/gpu_hl_ab.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --workload C2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-alt > gpurun_out/bench_C2.json 2> gpurun_out/bench_C2.err || { tail -30 gpurun_out/bench_C2.err; exit 1; }
tail -1 gpurun_out/bench_C2.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', d['ms_per_step'], d['phase_ms'])"
bash tools/gpu_c5.sh | python -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('C5x1', d['ms_per_step'], d['host_ms_per_stage_rank0'], d['one_gpu'])" || exit 1
bash tools/gpu_hl_ab.sh l75
