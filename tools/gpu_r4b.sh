#!/bin/bash
# round 4 K2 A/B: the tile-local parse tests against each experiment library, then C4 bench phases for each
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for n in "$@"; do
  export G2N_LIB=$R/gfa2network_amd/_lib/exp_$n.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_diff.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "tile_local or decimal_id or maxsym_buckets_match or csr_output" > gpurun_out/r4b_t_$n.log 2>&1 || { echo "TESTS FAILED $n"; tail -30 gpurun_out/r4b_t_$n.log; exit 1; }
  echo "$n tests: $(tail -1 gpurun_out/r4b_t_$n.log)"
done
unset G2N_LIB
bash tools/gpu_exp.sh "$@"
