#!/bin/bash
# 8 gloo ranks on the box's one GPU, 10^8 edges, decimal and hashed names (general protocol), vs one GPU
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest -m gpu -x -v -s --timeout 1000 --timeout-method thread tests/test_gpu_shard_scale.py > gpurun_out/shard_8rank_1e8.log 2>&1 || { tail -40 gpurun_out/shard_8rank_1e8.log; exit 1; }
grep -E "PASSED|FAILED|decimal|hashed" gpurun_out/shard_8rank_1e8.log | tail -8
