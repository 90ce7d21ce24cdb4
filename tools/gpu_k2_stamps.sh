#!/bin/bash
# K2 phase stamps on C4: the -DG2N_K2_STAMPS variant (tools/exp_build.sh stamps "-DG2N_K2_STAMPS")
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
G2N_LIB=$R/gfa2network_amd/_lib/exp_${1:-stamps}.so G2N_K2_STAMPS_OUT=$R/gpurun_out/k2_stamps.bin \
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-e2e --no-cpu-baseline --no-alt > gpurun_out/k2_stamps.log 2>&1 || { tail -20 gpurun_out/k2_stamps.log; exit 1; }
python tools/k2_stamps.py gpurun_out/k2_stamps.bin gpurun_out/k2_stamps.json
rm -f gpurun_out/k2_stamps.bin
