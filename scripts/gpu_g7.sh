# round 4 A/B: assign at 7 / 8 waves per SIMD (launch bounds) vs the default 6
set -u
export TMPDIR=/tmp
O=gpurun_out/g7; mkdir -p $O
HQ_LIB_PATH=hybridquantization_amd/libhq_w8.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "assign or config3 or packed or grid_margin or golden or wide or chunked" > $O/pytest_w8.log 2>&1 || { echo "w8 tests failed"; tail -5 $O/pytest_w8.log; exit 1; }
tail -1 $O/pytest_w8.log
LIBS="libhq.so libhq_w8.so libhq_w7.so" BENCH_ARGS="--no-full-search --steps 100" bash scripts/gpu_libab.sh
for L in libhq.so libhq_w8.so; do
  HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search --shard-of 8 > $O/shard8_$L.json 2>> $O/err || exit $?
  python3 -c "import json; d=json.load(open('$O/shard8_$L.json')); print('$L shard8', d['ms_per_step'], d['kernel_avg_ms'])"
done
