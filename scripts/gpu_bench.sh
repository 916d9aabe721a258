# Round-end style run: GPU tests, smoke, bench JSON, and rocprofv3 kernel-trace stats of the bench.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/bench
stop_if_fatal() { if [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; then echo "fatal rc=$1 at $2"; exit "$1"; fi; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/bench/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/bench/pytest_gpu.log; stop_if_fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/bench/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/bench/smoke.log; stop_if_fatal $rc smoke
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench/bench.json 2> gpurun_out/bench/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench/bench.json; tail -3 gpurun_out/bench/bench.err; stop_if_fatal $rc bench
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/bench/rocprof -o bench -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench/bench_rocprof.json 2> gpurun_out/bench/bench_rocprof.err
rc=$?; echo "rocprof rc=$rc"; cat gpurun_out/bench/bench_rocprof.json; stop_if_fatal $rc rocprof
cut -c1-160 gpurun_out/bench/rocprof/bench_kernel_stats.csv | head -8
exit 0
