#!/bin/bash
# the sharded GPU suites (gloo world 2/3 general protocol through the new ranking kernels), then the
# sharded protocol at N = 1 on C4 (hashed names forced through the general protocol; decimal)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -X faulthandler -m pytest -m gpu -x -v --timeout 170 --timeout-method thread \
  tests/test_gpu_shard.py tests/test_gpu_shard_scale.py > gpurun_out/r4j_tests.log 2>&1 || { tail -60 gpurun_out/r4j_tests.log; exit 1; }
tail -2 gpurun_out/r4j_tests.log
bash tools/gpu_shard_x1.sh
