# GPU suite + smoke + one default bench line on one box, each step bounded.
# Output: gpurun_out/chk/.  BENCH_ARGS: extra bench.py arguments.
set -u
export TMPDIR=/tmp
O=gpurun_out/chk; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --durations=15 --timeout 240 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 $O/bench.json; exit $rc
