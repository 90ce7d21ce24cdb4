#!/bin/bash
# F1w one sorting network per wave: weighted parity tests + the C3 leg (x2) + its kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -X faulthandler -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_diff.py -k "weighted_sum or csr_output" tests/test_gpu_fullsize.py::test_c3_full_size_equals_oracle \
  > gpurun_out/r4s_tests.log 2>&1 || { tail -80 gpurun_out/r4s_tests.log; exit 1; }
tail -2 gpurun_out/r4s_tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --workload C3 --steps 30 --warmup 3 --no-e2e --no-cpu-baseline --no-alt > gpurun_out/r4s_c3.json 2> gpurun_out/r4s_c3.err || { tail -30 gpurun_out/r4s_c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r4s_c3.json').read().splitlines()[-1]); print('C3', d['ms_per_step'], d['device_ms_per_step'], d['phase_ms'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3s -o run -- python3 $R/bench.py --workload C3 --steps 5 --warmup 1 --no-e2e --no-alt --no-cpu-baseline > $R/gpurun_out/r4s_prof.log 2>&1 || { tail -30 $R/gpurun_out/r4s_prof.log; exit 1; }
python3 $R/tools/rocpd_stats.py $R/gpurun_out/prof_c3s/run_results.db 14
