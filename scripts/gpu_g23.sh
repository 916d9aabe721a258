# rocprofv3 kernel-trace stats of the default bench line and the HBM traffic
# passes, on the tree with per-wave cost partials.  Output: gpurun_out/g23/.
set -u
export TMPDIR=/tmp
E=gpurun_out/g23
mkdir -p $E
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $E/trace -o bench -- python3 bench.py --no-cpu-baseline > $E/bench_under_rocprof.json 2> $E/bench_under_rocprof.err || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "cost|assign|build_grid|sa_step|finalize" -f csv -d $E/traffic_$c -o run -- python3 scripts/profile_eval.py --evals 3 > $E/traffic_$c.log 2>&1 || exit $?
done
