# Same-box A/B of ab/libhq_old.so vs ab/libhq_new.so over several bench shapes
# (one line per shape and library: ms per step, assign kernel ms).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/abm
i=0
for shape in "--size 1024 --K 64 --population 1 --steps 200" "--size 4096 --shard-of 8 --steps 100" \
             "--size 4096 --shard-of 8 --population 1 --steps 100" "--size 2048 --steps 100"; do
  i=$((i+1))
  for v in old new old new; do
    HQ_LIB_PATH=ab/libhq_$v.so timeout -k 10 120 python bench.py --no-cpu-baseline $shape > gpurun_out/abm/$v$i.json 2> gpurun_out/abm/$v$i.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "$v$i rc=$rc"; tail -3 gpurun_out/abm/$v$i.err; exit $rc; fi
    python3 -c "
import json;d=json.load(open('gpurun_out/abm/$v$i.json'))
print('$i $v', d['ms_per_step'], d['kernel_avg_ms']['assign'])"
  done
done
