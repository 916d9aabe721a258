set -u
mkdir -p gpurun_out/g1
timeout -k 10 120 ./scripts/mbs > gpurun_out/g1/mbs.txt 2>&1; rc=$?; cat gpurun_out/g1/mbs.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search --steps 100 > gpurun_out/g1/bench.json 2> gpurun_out/g1/bench.err; rc=$?; cut -c1-300 gpurun_out/g1/bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search --shard-of 8 --steps 200 > gpurun_out/g1/shard8.json 2> gpurun_out/g1/shard8.err; rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/g1/shard8.json')); print(d['ms_per_step'], d['kernel_avg_ms'])"
exit $rc
