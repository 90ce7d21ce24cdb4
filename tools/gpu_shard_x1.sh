#!/bin/bash
# The sharded protocol at N = 1 on C4 with hashed segment names: forced general protocol vs the
# single-GPU hash-tier build of the same bytes (bench line's one_gpu), and the decimal fast path.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --shard --workload C4 --names hashed --force-protocol --steps 3 --warmup 1 > gpurun_out/shard_x1_hashed_forced.json 2> gpurun_out/shard_x1_hashed_forced.err || { tail -30 gpurun_out/shard_x1_hashed_forced.err; exit 1; }
tail -1 gpurun_out/shard_x1_hashed_forced.json
timeout -k 10 400 python -u bench.py --shard --workload C4 --steps 3 --warmup 1 > gpurun_out/shard_x1_dec.json 2> gpurun_out/shard_x1_dec.err || { tail -30 gpurun_out/shard_x1_dec.err; exit 1; }
tail -1 gpurun_out/shard_x1_dec.json
