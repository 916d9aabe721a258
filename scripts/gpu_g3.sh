# round 4: chunked K > 256 path -- GPU tests, then bench lines (K=1024 device loop, default, shard-of-8)
set -u
export TMPDIR=/tmp
O=gpurun_out/g3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "device_search or wide or chunked or nonfinite or golden or search" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" $O/pytest.log | tail -5; [ $rc -ne 0 ] && exit $rc
for cfg in "--size 1024 --K 1024 --steps 50 --warmup 5" "--size 1024 --K 256 --steps 50 --warmup 5" ""; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search $cfg >> $O/configs.jsonl 2>> $O/configs.err
  rc=$?; echo "config [$cfg] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 -c "
import json
for l in open('$O/configs.jsonl'):
    d=json.loads(l); r=d['roofline']; print(d['ms_per_step'], d['value'], r['kernel'], d.get('kernel_avg_ms'), r['frac'])"
exit 0
