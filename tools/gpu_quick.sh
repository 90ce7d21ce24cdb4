#!/bin/bash
# GPU tests (optionally a -k filter) then a short C4 bench with phases; each step under its own limit
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
fi
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-e2e --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phase_ms'], d.get('alt_paths',{}).get('hash_dictionary',{}).get('ms_per_step'))"
