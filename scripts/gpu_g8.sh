# round 4 A/B: assign candidate walk on u32 keys (+ list padding), used colours as
# LDS bytes, occupancy 7/8 waves; the full GPU suite on the padded-key build first
set -u
export TMPDIR=/tmp
O=gpurun_out/g8; mkdir -p $O
HQ_LIB_PATH=hybridquantization_amd/libhq_k2.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_k2.log 2>&1 || { echo "k2 tests failed"; tail -30 $O/pytest_k2.log; exit 1; }
tail -1 $O/pytest_k2.log
HQ_LIB_PATH=hybridquantization_amd/libhq_k1.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "assign or config3 or packed or grid_margin or golden or chunked or pixel" > $O/pytest_k1.log 2>&1 || { echo "k1 tests failed"; tail -30 $O/pytest_k1.log; exit 1; }
tail -1 $O/pytest_k1.log
LIBS="libhq.so libhq_ub.so libhq_k1.so libhq_k2.so libhq_k2w7.so libhq_k2w8.so" BENCH_ARGS="--no-full-search --steps 100" bash scripts/gpu_libab.sh || exit $?
for L in libhq.so libhq_k2.so libhq_k2w8.so; do
  HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --shard-of 8 --steps 200 > $O/shard8_$L.json 2>> $O/err || exit $?
  python3 -c "import json; d=json.load(open('$O/shard8_$L.json')); print('$L shard8', d['ms_per_step'], d['kernel_avg_ms'])"
done
