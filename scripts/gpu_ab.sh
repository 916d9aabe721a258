# Same-box A/B of bench variants: each line of $VARIANTS (';'-separated option lists,
# e.g. "cost_rows=8;cost_rows=16") runs bench.py twice, alternating; one JSON per run.
set -u
mkdir -p gpurun_out/ab
i=0
for rep in 1 2; do
  IFS=';' read -ra VS <<< "$VARIANTS"
  for v in "${VS[@]}"; do
    i=$((i+1)); opts=""
    for kv in $v; do opts="$opts --opt $kv"; done
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-100} $opts ${BENCH_ARGS:-} > gpurun_out/ab/run$i.json 2> gpurun_out/ab/run$i.err
    rc=$?
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/run$i.json')); print('$v', d['value'], d['ms_per_step'], d['kernel_avg_ms'])" || { echo "rc=$rc"; tail -5 gpurun_out/ab/run$i.err; }
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  done
done
