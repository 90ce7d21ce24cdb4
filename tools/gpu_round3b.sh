#!/bin/bash
# Round-3 follow-up: the synthetic parity tests (incl. far links), C2 / C3 legs + kernel stats, the
# sharded C5 line at world 1 and the forced general protocol at N = 1 on C4 (hashed names)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_diff.py -m gpu -x -q -k "synthetic" --timeout 300 --timeout-method thread > gpurun_out/t_synth.log 2>&1 || { tail -30 gpurun_out/t_synth.log; exit 1; }
tail -2 gpurun_out/t_synth.log
for W in C3 C2; do
  timeout -k 10 300 python bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/bench_$W.json 2> gpurun_out/bench_$W.err || { tail -30 gpurun_out/bench_$W.err; exit 1; }
  BENCH_ARGS="--workload $W" bash tools/gpu_prof.sh prof_$W || exit 1
done
bash tools/gpu_c5.sh || exit 1
bash tools/gpu_shard_x1.sh
