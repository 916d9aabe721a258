# round 4: per-pixel dE parity, packed-image tests, assign quad A/B, bench roofline lines
set -u
export TMPDIR=/tmp
O=gpurun_out/g2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -rP -k "pixel_errors or packed_image or golden or fast_path or wide_palette_vs or assign or adversarial or clustered or special or config3 or grid_margin or workgroup" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" $O/pytest.log | tail -5; [ $rc -ne 0 ] && exit $rc
for q in 1 0 1 0; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search --steps 50 --opt assign_quad=$q >> $O/ab.jsonl 2>> $O/ab.err
  rc=$?; echo "quad $q rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
for cfg in "" "--dpi 96 --distance 60" "--size 1024 --K 1024 --steps 10 --warmup 2"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search $cfg >> $O/configs.jsonl 2>> $O/configs.err
  rc=$?; echo "config [$cfg] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search --shard-of 8 > $O/shard8.json 2> $O/shard8.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --no-full-search --steps 50 > $O/bench_rocprof.json 2> $O/bench_rocprof.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8 -o run -- python3 bench.py --no-cpu-baseline --no-full-search --shard-of 8 --steps 100 > $O/shard8_rocprof.json 2> $O/shard8_rocprof.err || exit $?
timeout -k 10 120 ./scripts/mbs > $O/mbs.txt || exit $?
python3 -c "
import json
for f in ['$O/ab.jsonl', '$O/configs.jsonl', '$O/shard8.json']:
    for l in open(f):
        d=json.loads(l); r=d['roofline']; print(f, d['ms_per_step'], d['value'], r['kernel'], r.get('kernel_avg_ms'), d.get('kernel_avg_ms'), r['frac'], r['frac_executed_taps'])"
exit 0
