# A/B of two library builds on one box: ab/libhq_old.so vs ab/libhq_new.so, alternated
# $REPS times, bench.py with $BENCH_ARGS (HQ_LIB_PATH selects the library).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for i in $(seq 1 ${REPS:-3}); do
  for v in old new; do
    HQ_LIB_PATH=ab/libhq_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab/$v$i.json 2> gpurun_out/ab/$v$i.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "$v$i rc=$rc"; tail -3 gpurun_out/ab/$v$i.err; exit $rc; fi
    python3 -c "
import json;d=json.loads(open('gpurun_out/ab/$v$i.json').read().strip().splitlines()[-1])
print('$v', d['ms_per_step'], d['kernel_avg_ms'])"
  done
done
