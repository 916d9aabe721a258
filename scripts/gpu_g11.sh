# A/B: LabRef read with non-temporal loads in cost16w (keeps the packed image in
# the MALL for the next assign?)
set -u
export TMPDIR=/tmp
O=gpurun_out/g11; mkdir -p $O
HQ_LIB_PATH=hybridquantization_amd/libhq_labnt.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "config3 or golden or pixel" > $O/pytest_labnt.log 2>&1 || { echo "labnt tests failed"; tail -20 $O/pytest_labnt.log; exit 1; }
tail -1 $O/pytest_labnt.log
LIBS="libhq.so libhq_labnt.so" BENCH_ARGS="--no-full-search --steps 100" bash scripts/gpu_libab.sh || exit $?
for L in libhq.so libhq_labnt.so; do
  HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --shard-of 8 --steps 200 > $O/shard8_$L.json 2>> $O/err || exit $?
  python3 -c "import json; d=json.load(open('$O/shard8_$L.json')); print('$L shard8', d['ms_per_step'], d['kernel_avg_ms'])"
  HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --population 64 --steps 10 --warmup 5 > $O/c5_$L.json 2>> $O/err || exit $?
  python3 -c "import json; d=json.load(open('$O/c5_$L.json')); print('$L C5', d['ms_per_step'], d['kernel_avg_ms'])"
done
