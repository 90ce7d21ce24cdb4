#!/bin/bash
# the rest of the -m gpu suite after test_gpu_fullsize's int64 test, then the C5 line at world 1
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -X faulthandler -m pytest -m gpu -x -v --timeout 170 --timeout-method thread \
  tests/test_gpu_fullsize.py::test_int64_indices_past_2_31_entries tests/test_gpu_golden.py tests/test_gpu_gzip_prefix.py \
  tests/test_gpu_hash_lean.py tests/test_gpu_ingest.py tests/test_gpu_shard.py tests/test_gpu_shard_scale.py \
  tests/test_split_golden.py > gpurun_out/r4g_tests.log 2>&1 || { tail -60 gpurun_out/r4g_tests.log; exit 1; }
tail -2 gpurun_out/r4g_tests.log
timeout -k 10 170 python -u bench.py --gpus 1 --workload C5 --shard --steps 5 --warmup 2 > gpurun_out/r4g_c5.log 2>&1 || { tail -30 gpurun_out/r4g_c5.log; exit 1; }
tail -1 gpurun_out/r4g_c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5x1', d['ms_per_step'], d['host_ms_per_stage_rank0'], d['one_gpu'])"
