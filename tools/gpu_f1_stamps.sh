#!/bin/bash
# F1 (k_sym_finish / k_sumw_finish) phase stamps: the -DG2N_F1_STAMPS variant (tools/exp_build.sh f1st
# "-DG2N_F1_STAMPS"); C4 by default, BENCH_ARGS="--workload C3 --no-c5-reference" for F1w
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
G2N_LIB=$R/gfa2network_amd/_lib/exp_${1:-f1st}.so G2N_F1_STAMPS_OUT=$R/gpurun_out/f1_stamps.bin \
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-e2e --no-cpu-baseline --no-alt $BENCH_ARGS > gpurun_out/f1_stamps.log 2>&1 || { tail -20 gpurun_out/f1_stamps.log; exit 1; }
python tools/k2_stamps.py gpurun_out/f1_stamps.bin gpurun_out/f1_stamps.json f1
rm -f gpurun_out/f1_stamps.bin
