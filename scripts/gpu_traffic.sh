# HBM traffic per launch of the default cost/assign kernels: separate FETCH_SIZE and
# WRITE_SIZE passes (MI355X_MICROARCH.md, HBM), summarised by scripts/pmc_traffic.py.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "cost_|assign|build_grid" -f csv -d gpurun_out/traffic/fetch -o run -- python3 scripts/profile_eval.py --evals 3 > gpurun_out/traffic/fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "cost_|assign|build_grid" -f csv -d gpurun_out/traffic/write -o run -- python3 scripts/profile_eval.py --evals 3 > gpurun_out/traffic/write.log 2>&1
rc=$?; echo "write rc=$rc"; exit $rc
