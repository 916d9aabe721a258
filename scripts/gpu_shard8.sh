set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/sat
timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --shard-of 8 --steps 200 > gpurun_out/sat/shard8.json 2> gpurun_out/sat/shard8.err || exit $?
cat gpurun_out/sat/shard8.json
HQ_LIB_PATH=hybridquantization_amd/libhq_sat.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --shard-of 8 --steps 20 > gpurun_out/sat/sat.json 2> gpurun_out/sat/sat.err || exit $?
grep -c SA_T gpurun_out/sat/sat.json || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/sat/trace -o run -- python3 bench.py --no-cpu-baseline --no-full-search --shard-of 8 --steps 200 > gpurun_out/sat/trace.log 2>&1 || exit $?
find gpurun_out/sat/trace -name "*stats*"
