# GPU tests selected by $TESTK (all when empty), then bench.py (no CPU baseline) with $BENCH_ARGS
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/tb
stop_if_fatal() { if [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; then echo "fatal rc=$1 at $2"; exit "$1"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTK:+-k "$TESTK"} > gpurun_out/tb/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/tb/pytest.log; stop_if_fatal $rc pytest
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/tb/bench.json 2> gpurun_out/tb/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-330 gpurun_out/tb/bench.json; tail -3 gpurun_out/tb/bench.err; stop_if_fatal $rc bench
exit 0
