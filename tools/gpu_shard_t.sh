#!/bin/bash
# the sharded GPU tests (gloo world 2/3 on one GPU, RCCL world 1, 8 ranks at 10^8 edges) and the C5 line at world 1
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_shard_scale.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t_shard.log 2>&1 || { tail -40 gpurun_out/t_shard.log; exit 1; }
tail -2 gpurun_out/t_shard.log
bash tools/gpu_c5.sh | python -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('C5x1', d['ms_per_step'], d['host_ms_per_stage_rank0'], d['one_gpu'])"
