# GPU check: parity tests ($TESTK selects), smoke, bench ($BENCH_ARGS), each bounded.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ck
stop_if_fatal() { if [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; then echo "fatal rc=$1 at $2"; exit "$1"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -rA --durations=0 ${TESTK:+-k "$TESTK"} > gpurun_out/ck/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/ck/pytest.log | tail -5; stop_if_fatal $rc pytest
[ $rc -ne 0 ] && exit $rc
[ -n "${SKIP_SMOKE:-}" ] || { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ck/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/ck/smoke.log; stop_if_fatal $rc smoke; [ $rc -ne 0 ] && exit $rc; }
[ -n "${SKIP_BENCH:-}" ] && exit 0
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/ck/bench.json 2> gpurun_out/ck/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/ck/bench.json; tail -3 gpurun_out/ck/bench.err; stop_if_fatal $rc bench
exit $rc
