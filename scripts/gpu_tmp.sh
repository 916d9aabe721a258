set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/g6
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "hrow4 or geometry or pixel_errors or generic or wide_palette or chunked" > gpurun_out/g6/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/g6/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="vt2=libhq.so:gen_vmfma=0;vm=libhq.so:gen_vmfma=1;vm8=libhq.so:gen_vmfma=1,gen_hrow_outputs=8" BENCH_ARGS="--dpi 300 --distance 50 --no-full-search --steps 10 --warmup 3" bash scripts/gpu_ab.sh || exit $?
VARIANTS="k8192=libhq.so:" BENCH_ARGS="--size 1024 --K 8192 --steps 5 --warmup 2 --no-full-search" REPS=1 bash scripts/gpu_ab.sh || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/g6/trace -o run -- python3 bench.py --no-cpu-baseline --no-full-search --dpi 300 --distance 50 --steps 10 --warmup 3 > gpurun_out/g6/trace.json 2>&1
rc=$?; echo "trace rc=$rc"; find gpurun_out/g6/trace -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160 | head -4
