# Same-box sweep of one hq_set_option ($OPT over $VALS) on bench.py ($BENCH_ARGS), twice each.
set -u
mkdir -p gpurun_out/sweep
for rep in 1 2; do
  for v in $VALS; do
    timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} --opt $OPT=$v > gpurun_out/sweep/$v.$rep.json 2> gpurun_out/sweep/$v.$rep.err
    rc=$?
    python3 -c "import json; d=json.load(open('gpurun_out/sweep/$v.$rep.json')); print('$OPT=$v', d['ms_per_step'], d['value'])" || { echo "$v rc=$rc"; tail -3 gpurun_out/sweep/$v.$rep.err; }
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  done
done
