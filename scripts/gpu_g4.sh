# round 4 A/B: scalar horizontal FMAs (libhq_hs) and integer cell of packed pixels (libhq_ci) vs base
set -u
export TMPDIR=/tmp
O=gpurun_out/g4; mkdir -p $O
HQ_LIB_PATH=hybridquantization_amd/libhq_ci.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "assign or config3 or packed or grid_margin or golden" > $O/pytest_ci.log 2>&1 || { echo "ci tests failed"; tail -5 $O/pytest_ci.log; exit 1; }
HQ_LIB_PATH=hybridquantization_amd/libhq_hs.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "golden or fast_path or pixel_errors" > $O/pytest_hs.log 2>&1 || { echo "hs tests failed"; tail -5 $O/pytest_hs.log; exit 1; }
tail -1 $O/pytest_ci.log $O/pytest_hs.log
LIBS="libhq.so libhq_hs.so libhq_ci.so" BENCH_ARGS="--no-full-search --steps 100" bash scripts/gpu_libab.sh
timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search --shard-of 8 > $O/shard8.json 2> $O/shard8.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search --size 1024 --K 1024 > $O/k1024.json 2> $O/k1024.err || exit $?
python3 -c "import json; [print(f, json.load(open(f))[\"ms_per_step\"], json.load(open(f))[\"kernel_avg_ms\"]) for f in [\"$O/shard8.json\", \"$O/k1024.json\"]]"
