#!/bin/bash
# output-centric decimal names: name parity (decimal tiers, goldens, full-size digests), then C4 A/B
# against the byte-store form (nbytes) on the same box
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -X faulthandler -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_diff.py -k "decimal or tile_local or synthetic or c4_prop" tests/test_gpu_golden.py \
  tests/test_gpu_fullsize.py::test_c4_full_size_equals_oracle tests/test_gpu_fullsize.py::test_c2_full_size_equals_oracle \
  tests/test_gpu_fullsize.py::test_c3_full_size_equals_oracle \
  > gpurun_out/r4u_tests.log 2>&1 || { tail -80 gpurun_out/r4u_tests.log; exit 1; }
tail -2 gpurun_out/r4u_tests.log
for rep in 1 2; do
for v in default nbytes; do
  if [ $v = default ]; then unset G2N_LIB; else export G2N_LIB=$R/gfa2network_amd/_lib/exp_$v.so; fi
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --no-alt > gpurun_out/r4u_$v.json 2> gpurun_out/r4u_$v.err || { tail -20 gpurun_out/r4u_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4u_$v.json').read().splitlines()[-1]); print('$v', d['ms_per_step'], d.get('phase_ms'))"
done
done
unset G2N_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4u -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-e2e --no-alt --no-cpu-baseline > $R/gpurun_out/r4u_prof.log 2>&1 || { tail -30 $R/gpurun_out/r4u_prof.log; exit 1; }
python3 $R/tools/rocpd_stats.py $R/gpurun_out/prof_c4u/run_results.db 10
