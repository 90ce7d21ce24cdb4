#!/bin/bash
# K2 tile shape A/B: 16 KiB tiles (512 threads, 2 chunks each; or 256 threads, 4 chunks) against 32 KiB
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in t16 t16w4; do
  G2N_LIB=$R/gfa2network_amd/_lib/exp_$v.so timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_fullsize.py::test_c4_full_size_equals_oracle tests/test_gpu_diff.py -k "tile_local or decimal_id" > gpurun_out/r4t16_$v.log 2>&1 || { tail -30 gpurun_out/r4t16_$v.log; exit 1; }
  tail -1 gpurun_out/r4t16_$v.log
done
for rep in 1 2; do
for v in default t16 t16w4; do
  if [ $v = default ]; then unset G2N_LIB; else export G2N_LIB=$R/gfa2network_amd/_lib/exp_$v.so; fi
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --no-alt > gpurun_out/r4t16_$v.json 2> gpurun_out/r4t16_$v.err || { tail -20 gpurun_out/r4t16_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4t16_$v.json').read().splitlines()[-1]); print('$v', d['ms_per_step'], d.get('phase_ms'))"
done
done
