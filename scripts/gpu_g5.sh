# round 4: fixed-point dE sums + fused SA step / grid launch -- GPU suite, A/B sa_fuse, shard-of-8
set -u
export TMPDIR=/tmp
O=gpurun_out/g5; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" $O/pytest.log | tail -5; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for f in 1 0; do
  for cfg in "" "--shard-of 8"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search --opt sa_fuse=$f $cfg >> $O/ab.jsonl 2>> $O/ab.err
    rc=$?; echo "fuse $f [$cfg] rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done; done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search --size 1024 --K 1024 >> $O/ab.jsonl 2>> $O/ab.err || exit $?
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['ms_per_step'], d['value'], d['config'].get('options'), d['config'].get('shard_of'), d.get('kernel_avg_ms'))"
exit 0
