# cost16w ablations (wrong results, timing only) of the stripped kernel (no memory
# loads, gathers, Lab/dE or horizontal taps): without the vertical stores, without
# the MFMA and its operand packing, without the reduction, without all three
set -u
export TMPDIR=/tmp
LIBS="libhq.so libhq_s_nomem.so libhq_s_novst.so libhq_s_nomfma.so libhq_s_nored2.so libhq_s_none.so" BENCH_ARGS="--no-full-search --steps 100" bash scripts/gpu_libab.sh
