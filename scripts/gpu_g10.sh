# cost16w ablations (wrong results, timing only) on the stripped kernel (no
# gathers, Lab/dE or horizontal taps: fill, MFMA, stores, barriers): without its
# fill loads, without the LabRef loads, without both, + one MFMA product; and the
# full kernel without its fill loads
set -u
export TMPDIR=/tmp
LIBS="libhq.so libhq_nogatlh.so libhq_s_nofill.so libhq_s_nolabld.so libhq_s_nomem.so libhq_s_nomemv.so libhq_nofill.so" BENCH_ARGS="--no-full-search --steps 100" bash scripts/gpu_libab.sh
