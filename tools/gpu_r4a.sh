#!/bin/bash
# round 4: the new parity tests (C2 at config size, call state after a failed build, int64 index path,
# sharded tile-local range premise / one-pass protocol) + the sharded suites, then the C5 line at world 1
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 800 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py::test_c2_full_size_equals_oracle tests/test_gpu_diff.py::test_failed_build_leaves_no_call_state \
  tests/test_gpu_diff.py::test_int64_index_path_equals_oracle tests/test_gpu_shard.py tests/test_gpu_shard_scale.py \
  tests/test_gpu_fullsize.py::test_int64_indices_past_2_31_entries > gpurun_out/r4a_tests.log 2>&1 || { tail -60 gpurun_out/r4a_tests.log; exit 1; }
tail -3 gpurun_out/r4a_tests.log
bash tools/gpu_c5.sh | python -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('C5x1', d['ms_per_step'], d['host_ms_per_stage_rank0'], d['one_gpu'])"
