# round 4: LDS-tiled generic path -- GPU suite, then 300/50 and K=8192 lines: tiled (variant 1) vs per-pixel (variant 2)
set -u
export TMPDIR=/tmp
O=gpurun_out/g6; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" $O/pytest.log | tail -5; [ $rc -ne 0 ] && exit $rc
for v in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search --dpi 300 --distance 50 --steps 10 --warmup 2 --opt cost_variant=$v >> $O/configs.jsonl 2>> $O/configs.err || exit $?
  echo "300/50 variant $v ok"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search --dpi 96 --distance 60 >> $O/configs.jsonl 2>> $O/configs.err || exit $?
for ov in 1 0 1 0; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search --population 64 --steps 20 --warmup 5 --opt overlap=$ov >> $O/configs.jsonl 2>> $O/configs.err || exit $?
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search --population 8 >> $O/configs.jsonl 2>> $O/configs.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search --population 64 --shard-of 8 --steps 20 --warmup 5 >> $O/configs.jsonl 2>> $O/configs.err || exit $?
for L in libhq.so libhq_ns.so libhq.so libhq_ns.so; do
  for cfg in "--dpi 96 --distance 60" "--dpi 150 --distance 30"; do
    HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-full-search $cfg > $O/split_$L.json 2>> $O/configs.err || exit $?
    python3 -c "import json; d=json.load(open('$O/split_$L.json')); print('$L', '$cfg', d['ms_per_step'], d['kernel_avg_ms']['cost'])" | tee -a $O/split.txt
  done
done
python3 -c "
import json
for l in open('$O/configs.jsonl'):
    d=json.loads(l); r=d['roofline']; print(d['ms_per_step'], d['value'], r['kernel'], d.get('kernel_avg_ms'), r['frac'], d['config'].get('options'))"
exit 0
