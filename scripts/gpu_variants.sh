# Bench variants, one line each: VARIANTS is a ';'-separated list of bench.py argument sets.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/var
i=0
IFS=';' read -ra VS <<< "${VARIANTS}"
for v in "${VS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline $v > gpurun_out/var/v$i.json 2> gpurun_out/var/v$i.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "variant $i ($v) rc=$rc"; tail -3 gpurun_out/var/v$i.err; exit $rc; fi
  python3 -c "
import json,sys;d=json.loads(open('gpurun_out/var/v$i.json').read().strip().splitlines()[-1])
print('$v'.strip().ljust(60), d['ms_per_step'], d['value'], d['kernel_avg_ms'])"
done
