# Same-box A/B over (library, options) cases: $CASES = space-separated
# lib.so[:NAME=VALUE[,NAME=VALUE...]] items, each run twice (alternating) by
# bench.py with $BENCH_ARGS; one JSON per run under gpurun_out/matrix/.
set -u
mkdir -p gpurun_out/matrix
i=0
for rep in 1 2; do
  for c in $CASES; do
    i=$((i+1)); lib=${c%%:*}; opts=""
    if [ "$c" != "$lib" ]; then IFS=',' read -ra KV <<< "${c#*:}"; for kv in "${KV[@]}"; do opts="$opts --opt $kv"; done; fi
    HQ_LIB_PATH=hybridquantization_amd/$lib timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} $opts > gpurun_out/matrix/run$i.json 2> gpurun_out/matrix/run$i.err
    rc=$?
    python3 -c "import json; d=json.load(open('gpurun_out/matrix/run$i.json')); print('$c', d['ms_per_step'], d['value'], d['kernel_avg_ms'])" || { echo "$c rc=$rc"; tail -3 gpurun_out/matrix/run$i.err; }
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  done
done
