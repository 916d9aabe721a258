# Short vs long timed regions (the driver may time only a few steps); the full
# C3 search now runs before the timed loop
set -u
mkdir -p gpurun_out/steps
for k in 20 100; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps $k --warmup 5 > gpurun_out/steps/s$k.json 2> gpurun_out/steps/s$k.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/steps/s$k.json')); print($k, d['value'], d['ms_per_step'], d['kernel_avg_ms'], d['full_search_c3']['device_host_agree'])"
done
timeout -k 10 200 python bench.py --no-cpu-baseline --shard-of 8 --steps 100 --warmup 5 > gpurun_out/steps/shard8.json 2> gpurun_out/steps/shard8.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/steps/shard8.json')); print('shard8', d['value'], d['ms_per_step'], d['kernel_avg_ms'], d['full_search_c3']['ms_per_iteration_device'])"
