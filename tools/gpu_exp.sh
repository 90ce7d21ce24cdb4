#!/bin/bash
# C4 bench phases for each experiment library named on the command line (gfa2network_amd/_lib/exp_NAME.so)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
for n in base "$@"; do
  if [ "$n" != base ]; then export G2N_LIB=$R/gfa2network_amd/_lib/exp_$n.so; else unset G2N_LIB; fi
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-e2e --no-cpu-baseline --no-alt > gpurun_out/exp_$n.log 2>&1 || { tail -20 gpurun_out/exp_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/exp_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phase_ms'])")"
done
