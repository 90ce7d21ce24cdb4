#!/bin/bash
# The sharded C5 bench line on this box's one GPU (world 1 through torch.distributed.run), each step limited
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 1 --workload C5 --steps ${STEPS:-5} --warmup 2 > gpurun_out/bench_c5.log 2>&1 \
  || { tail -30 gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log
