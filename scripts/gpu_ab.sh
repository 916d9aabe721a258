# Same-box A/B of library builds and options, alternating, REPS rounds.
#   VARIANTS="label=lib.so:opt=v,opt=v;label2=lib2.so:"  (libs under hybridquantization_amd/)
#   BENCH_ARGS (default "--no-full-search --steps 200 --warmup 30"), REPS (default 2)
# One JSON per run under gpurun_out/ab/, one summary line per run on stdout.
set -u
mkdir -p gpurun_out/ab
IFS=';' read -ra VS <<< "$VARIANTS"
for rep in $(seq 1 ${REPS:-2}); do
  for v in "${VS[@]}"; do
    label=${v%%=*}; rest=${v#*=}; lib=${rest%%:*}; optstr=${rest#*:}
    opts=""; IFS=',' read -ra OS <<< "$optstr"; for kv in "${OS[@]}"; do [ -n "$kv" ] && opts="$opts --opt $kv"; done
    out=gpurun_out/ab/$label.$rep
    HQ_LIB_PATH=hybridquantization_amd/$lib timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:---no-full-search --steps 200 --warmup 30} $opts > $out.json 2> $out.err
    rc=$?
    python3 -c "import json; d=json.load(open('$out.json')); k=d['kernel_avg_ms']; print('$label', '$rep', d['value'], d['ms_per_step'], 'cost', k['cost'], 'assign', k['assign'], 'grid', k['grid'], 'sa', k['sa_step'])" || { echo "$label rc=$rc"; tail -3 $out.err; }
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
