#!/bin/bash
# round 4: the new parity tests (C2 at config size, call state after a failed build, int64 index path,
# sharded tile-local range premise / one-pass protocol) + the sharded suites, then the C5 line at world 1
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="python -u -X faulthandler -m pytest -x -v --timeout-method thread -m gpu"
timeout -k 10 200 $T --timeout 90 tests/test_gpu_diff.py::test_failed_build_leaves_no_call_state \
  tests/test_gpu_diff.py::test_int64_index_path_equals_oracle > gpurun_out/r4a_t1.log 2>&1 || { tail -80 gpurun_out/r4a_t1.log; exit 1; }
tail -2 gpurun_out/r4a_t1.log
timeout -k 10 600 $T --timeout 170 tests/test_gpu_shard.py > gpurun_out/r4a_t2.log 2>&1 || { tail -60 gpurun_out/r4a_t2.log; exit 1; }
tail -2 gpurun_out/r4a_t2.log
timeout -k 10 170 python -u bench.py --gpus 1 --workload C5 --shard --steps 5 --warmup 2 > gpurun_out/r4a_c5.log 2>&1 || { tail -30 gpurun_out/r4a_c5.log; exit 1; }
tail -1 gpurun_out/r4a_c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5x1', d['ms_per_step'], d['host_ms_per_stage_rank0'], d['one_gpu'])"
timeout -k 10 400 $T --timeout 170 tests/test_gpu_shard_scale.py tests/test_gpu_fullsize.py::test_int64_indices_past_2_31_entries > gpurun_out/r4a_t3.log 2>&1 || { tail -60 gpurun_out/r4a_t3.log; exit 1; }
tail -2 gpurun_out/r4a_t3.log
