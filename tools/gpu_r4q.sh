#!/bin/bash
# names kernel variant: name tests + C4 bench x2 + kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -X faulthandler -m pytest -m gpu -x -q --timeout 400 --timeout-method thread \
  tests/test_gpu_diff.py -k "decimal" tests/test_gpu_fullsize.py::test_c4_full_size_equals_oracle \
  > gpurun_out/r4q_tests.log 2>&1 || { tail -80 gpurun_out/r4q_tests.log; exit 1; }
tail -2 gpurun_out/r4q_tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --no-alt > gpurun_out/r4q_c4.json 2> gpurun_out/r4q_c4.err || { tail -30 gpurun_out/r4q_c4.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r4q_c4.json').read().splitlines()[-1]); print('C4', d['ms_per_step'], d.get('phase_ms'), d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4q -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-e2e --no-alt --no-cpu-baseline > $R/gpurun_out/r4q_prof.log 2>&1 || { tail -30 $R/gpurun_out/r4q_prof.log; exit 1; }
python3 $R/tools/rocpd_stats.py $R/gpurun_out/prof_c4q/run_results.db 8
