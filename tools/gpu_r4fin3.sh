#!/bin/bash
# F1 at 8 waves: the full-size digests, goldens and sharded suites
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -m gpu -x -q --timeout 400 --timeout-method thread \
  tests/test_gpu_fullsize.py tests/test_gpu_golden.py tests/test_gpu_shard.py > gpurun_out/r4fin3_tests.log 2>&1 || { tail -40 gpurun_out/r4fin3_tests.log; exit 1; }
tail -1 gpurun_out/r4fin3_tests.log
