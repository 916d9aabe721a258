# Same-box A/B of library builds: $LIBS = space-separated .so names under
# hybridquantization_amd/, each timed twice by bench.py (HQ_LIB_PATH override).
set -u
mkdir -p gpurun_out/libab
for rep in 1 2; do
  for L in $LIBS; do
    HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/libab/$L.$rep.json 2> gpurun_out/libab/$L.$rep.err
    rc=$?
    python3 -c "import json; d=json.load(open('gpurun_out/libab/$L.$rep.json')); print('$L', d['value'], d['kernel_avg_ms'])" || { echo "$L rc=$rc"; tail -3 gpurun_out/libab/$L.$rep.err; }
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  done
done
