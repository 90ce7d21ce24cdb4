#!/bin/bash
# the whole -m gpu suite (per-test limit, verbose so progress is visible), then the C5 line at world 1
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -X faulthandler -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1 || { tail -60 gpurun_out/r4f_tests.log; exit 1; }
tail -2 gpurun_out/r4f_tests.log
timeout -k 10 170 python -u bench.py --gpus 1 --workload C5 --shard --steps 5 --warmup 2 > gpurun_out/r4f_c5.log 2>&1 || { tail -30 gpurun_out/r4f_c5.log; exit 1; }
tail -1 gpurun_out/r4f_c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5x1', d['ms_per_step'], d['host_ms_per_stage_rank0'], d['one_gpu'])"
