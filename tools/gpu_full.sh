#!/bin/bash
# GPU test suite, then the driver's default bench command (C4 + alt paths + C2/C3 legs + CPU baseline + e2e)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['phase_ms'], d['roofline']['frac'], d.get('alt_paths',{}).get('hash_dictionary',{}).get('ms_per_step'))"
