#!/bin/bash
# the chunked single-GPU build (parse_gfa chunk_bytes) and the sharded suite
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -X faulthandler -m pytest -m gpu -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_shard.py > gpurun_out/r4w_tests.log 2>&1 || { tail -80 gpurun_out/r4w_tests.log; exit 1; }
tail -6 gpurun_out/r4w_tests.log
