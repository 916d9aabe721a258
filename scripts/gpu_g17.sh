# cost16w: LabRef loads issued earlier (HQ_LAB_EARLY 1: before channel 1's
# horizontal pass, 2: before channels 1-2's gathers) vs after channel 2's stores
# (0, default; base = the same before the refactor into a lambda)
set -u
export TMPDIR=/tmp
O=gpurun_out/g17; mkdir -p $O
HQ_LIB_PATH=hybridquantization_amd/libhq_le2.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "golden or config3 or pixel" > $O/pytest_le2.log 2>&1 || { echo "le2 tests failed"; tail -20 $O/pytest_le2.log; exit 1; }
tail -1 $O/pytest_le2.log
LIBS="libhq_base.so libhq.so libhq_le1.so libhq_le2.so" BENCH_ARGS="--no-full-search --steps 100" bash scripts/gpu_libab.sh
