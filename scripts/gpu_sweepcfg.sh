set -u
for cfg in "--size 1024 --K 64 --population 1 --steps 400 --warmup 100" "--population 1 --steps 200 --warmup 50" "--size 8192 --shard-of 8 --steps 200 --warmup 50" "--population 64 --steps 10 --warmup 10"; do
  echo "== $cfg"
  OPT=assign_blocks_per_cu VALS="8 16" BENCH_ARGS="--no-full-search $cfg" bash scripts/gpu_optsweep.sh || exit $?
done
