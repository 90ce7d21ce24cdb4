#!/bin/bash
# pair-word partition stream + F1w staging + protocol local builds without values: the partition /
# MAX-SYM / weighted / sharded parity tests, then C4 and C3 bench lines, the forced protocol at N = 1
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -X faulthandler -m pytest -m gpu -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_diff.py -k "maxsym or weighted_sum or csr_output or synthetic or int64 or failed_build or fuzz_gpu or c4_prop" \
  tests/test_gpu_fullsize.py::test_c4_full_size_equals_oracle tests/test_gpu_fullsize.py::test_c3_full_size_equals_oracle \
  tests/test_gpu_fullsize.py::test_c2_full_size_equals_oracle tests/test_gpu_shard.py \
  > gpurun_out/r4m_tests.log 2>&1 || { tail -80 gpurun_out/r4m_tests.log; exit 1; }
tail -3 gpurun_out/r4m_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-e2e --no-cpu-baseline > gpurun_out/r4m_c4.json 2> gpurun_out/r4m_c4.err || { tail -30 gpurun_out/r4m_c4.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r4m_c4.json').read().splitlines()[-1]); print('C4', d['ms_per_step'], d.get('phase_ms'), d['roofline']['frac'])"
timeout -k 10 300 python -u bench.py --workload C3 --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --no-alt > gpurun_out/r4m_c3.json 2> gpurun_out/r4m_c3.err || { tail -30 gpurun_out/r4m_c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r4m_c3.json').read().splitlines()[-1]); print('C3', d['ms_per_step'], d['device_ms_per_step'], d['phase_ms'])"
bash tools/gpu_shard_x1.sh
