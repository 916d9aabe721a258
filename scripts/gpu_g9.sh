# cost16w timing ablations (wrong results, timing only): no Opp->Lab/dE, no
# horizontal taps, one MFMA product instead of three; C3 and 96 dpi / 60 cm
set -u
export TMPDIR=/tmp
O=gpurun_out/g9; mkdir -p $O
LIBS="libhq.so libhq_nolab.so libhq_nohp.so libhq_mfma1.so libhq_nolabhp.so" BENCH_ARGS="--no-full-search --steps 100" bash scripts/gpu_libab.sh || exit $?
for L in libhq.so libhq_nolab.so libhq_nohp.so libhq_mfma1.so; do
  HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --dpi 96 --distance 60 > $O/d96_$L.json 2>> $O/err || exit $?
  python3 -c "import json; d=json.load(open('$O/d96_$L.json')); print('$L 96/60', d['ms_per_step'], d['kernel_avg_ms'])"
done
