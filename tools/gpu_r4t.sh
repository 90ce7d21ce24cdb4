#!/bin/bash
# quarter partition tiles below 2^24 elements + node names written by the tile-local parse: parity
# tests (partition, names, sharded), C2 / C3 legs, then C4 A/B against a build with k_names_dec (k2n0)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -X faulthandler -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_diff.py -k "weighted_sum or csr_output or maxsym or synthetic or int64_index or fuzz_gpu or convert_format or decimal or tile_local or failed_build" \
  tests/test_gpu_fullsize.py::test_c3_full_size_equals_oracle tests/test_gpu_fullsize.py::test_c2_full_size_equals_oracle \
  tests/test_gpu_fullsize.py::test_c4_full_size_equals_oracle tests/test_gpu_golden.py \
  tests/test_gpu_shard.py > gpurun_out/r4t_tests.log 2>&1 || { tail -80 gpurun_out/r4t_tests.log; exit 1; }
tail -2 gpurun_out/r4t_tests.log
for w in C3 C2; do
timeout -k 10 300 python -u bench.py --workload $w --steps 30 --warmup 3 --no-e2e --no-cpu-baseline --no-alt > gpurun_out/r4t_$w.json 2> gpurun_out/r4t_$w.err || { tail -30 gpurun_out/r4t_$w.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r4t_$w.json').read().splitlines()[-1]); print('$w', d['ms_per_step'], d['device_ms_per_step'], d['phase_ms'])"
done
for rep in 1 2; do
for v in default k2n0; do
  if [ $v = default ]; then unset G2N_LIB; else export G2N_LIB=$R/gfa2network_amd/_lib/exp_$v.so; fi
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --no-alt > gpurun_out/r4t_$v.json 2> gpurun_out/r4t_$v.err || { tail -20 gpurun_out/r4t_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4t_$v.json').read().splitlines()[-1]); print('$v', d['ms_per_step'], d.get('phase_ms'))"
done
done
