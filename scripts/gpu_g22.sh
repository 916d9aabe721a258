# bench.py after the accounting refactor: default line (CPU baseline, full search),
# 96/60, and cost_variant 2 (the per-pixel generic pair)
set -u
O=gpurun_out/g22; mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 > $O/b.json 2> $O/b.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --dpi 96 --distance 60 --steps 20 > $O/d96.json 2>> $O/b.err || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --steps 10 --opt cost_variant=2 > $O/v2.json 2>> $O/b.err || exit $?
python3 - <<'PY'
import json
for f in ("b", "d96", "v2"):
    d = json.load(open("gpurun_out/g22/" + f + ".json")); r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], r["kernel"], r["tap_bucket"], r["frac"], r.get("traffic"))
PY
