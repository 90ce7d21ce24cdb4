#!/bin/bash
# hash-dictionary leg of the C4 bench for base vs experiment libs
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
for n in base "$@"; do
  if [ "$n" != base ]; then export G2N_LIB=$R/gfa2network_amd/_lib/exp_$n.so; else unset G2N_LIB; fi
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline > gpurun_out/hl_$n.log 2>&1 || { tail -20 gpurun_out/hl_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/hl_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); h=d['alt_paths']['hash_dictionary']; print(d['ms_per_step'], h['ms_per_step'], h['phase_ms'])")"
done
