#!/bin/bash
# names by LDS-staged 16-byte stores: decimal-id name tests, C4 full-size digest, the C4 bench + kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -X faulthandler -m pytest -m gpu -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_diff.py -k "decimal or tile_local or synthetic or c4_prop" tests/test_gpu_golden.py \
  tests/test_gpu_fullsize.py::test_c4_full_size_equals_oracle tests/test_gpu_fullsize.py::test_c2_full_size_equals_oracle \
  tests/test_gpu_shard.py > gpurun_out/r4p_tests.log 2>&1 || { tail -80 gpurun_out/r4p_tests.log; exit 1; }
tail -3 gpurun_out/r4p_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --no-alt > gpurun_out/r4p_c4.json 2> gpurun_out/r4p_c4.err || { tail -30 gpurun_out/r4p_c4.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r4p_c4.json').read().splitlines()[-1]); print('C4', d['ms_per_step'], d.get('phase_ms'), d['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4p -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-e2e --no-alt --no-cpu-baseline > $R/gpurun_out/r4p_prof.log 2>&1 || { tail -30 $R/gpurun_out/r4p_prof.log; exit 1; }
python3 $R/tools/rocpd_stats.py $R/gpurun_out/prof_c4p/run_results.db 12
