#!/bin/bash
# the driver's bench (20 steps, e2e legs with their digests), the sharded protocol at N = 1 (hashed
# names forced through the general protocol; decimal fast path), then the tw2 A/B and the F1 stamps
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4h_bench.json 2> gpurun_out/r4h_bench.err || { tail -30 gpurun_out/r4h_bench.err; exit 1; }
tail -1 gpurun_out/r4h_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['phase_ms'], d['roofline']['frac'], {k: v.get('digest_ok') for k, v in d['end_to_end'].items() if isinstance(v, dict)}, d['alt_paths']['hash_dictionary']['ms_per_step'], {k: v['ms_per_step'] for k, v in d['other_configs'].items()})"
bash tools/gpu_shard_x1.sh || exit 1
bash tools/gpu_r4b.sh tw2 || exit 1
bash tools/gpu_f1_stamps.sh f1st && python -c "import json; d=json.load(open('gpurun_out/f1_stamps.json')); print({k: v for k, v in d.items() if k != 'per_cu'})"
