# quick GPU iteration: parity tests + eval timing (+ optional kernel trace)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
stop_if_fatal() { if [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; then echo "fatal rc=$1 at $2"; exit "$1"; fi; }
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=15 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
IFS=";" read -r -a cfgs <<< "${CFGS:---tile 4;--tile 2}"
for cfg in "${cfgs[@]}"; do
timeout -k 10 300 python scripts/profile_eval.py --evals 10 $cfg > gpurun_out/prof/eval_cfg.log 2>&1
rc=$?; cat gpurun_out/prof/eval_cfg.log; stop_if_fatal $rc eval
done
if [ "${1:-}" = "trace" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof/trace -o run -- python3 scripts/profile_eval.py --evals 10 > gpurun_out/prof/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; stop_if_fatal $rc trace
cut -c1-150 gpurun_out/prof/trace/run_kernel_stats.csv | head -8
fi
if [ "${2:-}" = "pmc" ]; then
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --kernel-include-regex "cost_tile|assign|build_grid" -f csv -d gpurun_out/prof/pmc$i -o run -- python3 scripts/profile_eval.py --evals 3 > gpurun_out/prof/pmc$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; stop_if_fatal $rc pmc$i
done
fi
exit 0
