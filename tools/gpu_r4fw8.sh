#!/bin/bash
# F1 at 8 waves per SIMD (G2N_FIN_W8: SGPRs capped, 34 spilled to VGPR lanes) against 7, same box
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
G2N_LIB=$R/gfa2network_amd/_lib/exp_fw8.so timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fullsize.py::test_c4_full_size_equals_oracle > gpurun_out/r4fw8_t.log 2>&1 || { tail -30 gpurun_out/r4fw8_t.log; exit 1; }
tail -1 gpurun_out/r4fw8_t.log
for rep in 1 2 3; do
for v in default fw8; do
  if [ $v = default ]; then unset G2N_LIB; else export G2N_LIB=$R/gfa2network_amd/_lib/exp_$v.so; fi
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --no-alt > gpurun_out/r4fw8_$v.json 2> gpurun_out/r4fw8_$v.err || { tail -20 gpurun_out/r4fw8_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4fw8_$v.json').read().splitlines()[-1]); print('$v', d['ms_per_step'], d.get('phase_ms'))"
done
done
