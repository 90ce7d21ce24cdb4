#!/bin/bash
# pass 7 staging its words as u32 (default) against the uint2 staging (p7old = HEAD), same box
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for rep in 1 2 3; do
for v in default p7old; do
  if [ $v = default ]; then unset G2N_LIB; else export G2N_LIB=$R/gfa2network_amd/_lib/exp_$v.so; fi
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --no-alt > gpurun_out/r4v_$v.json 2> gpurun_out/r4v_$v.err || { tail -20 gpurun_out/r4v_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4v_$v.json').read().splitlines()[-1]); print('$v', d['ms_per_step'], d.get('phase_ms'))"
done
done
