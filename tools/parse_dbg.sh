# Parse-kernel cost breakdown (G2N_PARSE_DBG bits skip parts of K2; the build stops after K2).
mkdir -p gpurun_out
for D in 0 1 2 4 8 12; do
  G2N_PARSE_DBG=$D timeout -k 10 120 python bench.py --no-e2e --no-cpu-baseline --no-alt --steps 3 --warmup 1 > gpurun_out/dbg_$D.json 2>&1 || exit 1
done
