#!/bin/bash
# phase stamps of the hash edge pass (k_tile_lean kLeanEdges) on C4 with hashed names:
# the -DG2N_K2_STAMPS variant (tools/exp_build.sh stamps "-DG2N_K2_STAMPS")
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
G2N_LIB=$R/gfa2network_amd/_lib/exp_${1:-stamps}.so G2N_HL_STAMPS_OUT=$R/gpurun_out/hl_stamps.bin \
  timeout -k 10 300 python -u bench.py --names hashed --steps 1 --warmup 1 --no-e2e --no-cpu-baseline --no-alt > gpurun_out/hl_stamps.log 2>&1 || { tail -20 gpurun_out/hl_stamps.log; exit 1; }
python tools/k2_stamps.py gpurun_out/hl_stamps.bin gpurun_out/hl_stamps.json
rm -f gpurun_out/hl_stamps.bin
