#!/bin/bash
# F1w with register-loaded elements + staged output: weighted parity tests, the C3 leg and its
# kernel stats; the sharded suites (local builds without values) and the forced protocol at N = 1
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -X faulthandler -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_diff.py -k "weighted_sum or csr_output or convert_format or float_duplicate or synthetic" \
  tests/test_gpu_fullsize.py::test_c3_full_size_equals_oracle tests/test_gpu_shard.py \
  > gpurun_out/r4l_tests.log 2>&1 || { tail -80 gpurun_out/r4l_tests.log; exit 1; }
tail -3 gpurun_out/r4l_tests.log
timeout -k 10 300 python -u bench.py --workload C3 --steps 20 --warmup 3 --no-e2e > gpurun_out/r4l_c3.json 2> gpurun_out/r4l_c3.err || { tail -30 gpurun_out/r4l_c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r4l_c3.json').read().splitlines()[-1]); print(d['ms_per_step'], d['device_ms_per_step'], d['phase_ms'])"
bash tools/gpu_shard_x1.sh
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3l -o run -- python3 $R/bench.py --workload C3 --steps 5 --warmup 1 --no-e2e --no-alt --no-cpu-baseline > $R/gpurun_out/r4l_prof.log 2>&1 || { tail -30 $R/gpurun_out/r4l_prof.log; exit 1; }
python3 $R/tools/rocpd_stats.py $R/gpurun_out/prof_c3l/run_results.db 14
