# Round evidence on one box, each step bounded and chained: GPU tests, smoke, the
# default bench line (CPU baseline + full C3 search), its rocprofv3 kernel-trace
# stats, HBM traffic passes, PMC passes of the cost and assign kernels, every
# BASELINE config, and the shard-of-8 per-rank step.  Output: gpurun_out/ev/.
# (The configs run before the counter passes: a line right after a PMC pass ran
# on clocks that had not settled.)
set -u
export TMPDIR=/tmp
E=gpurun_out/ev
mkdir -p $E
fatal() { if [ "$1" -ne 0 ]; then echo "FAILED rc=$1 at $2"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rA --durations=0 --timeout 300 --timeout-method thread -p no:cacheprovider > $E/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $E/pytest_gpu.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $E/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $E/smoke.log; fatal $rc smoke
timeout -k 10 600 python bench.py > $E/bench.json 2> $E/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 $E/bench.json; fatal $rc bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $E/trace -o bench -- python3 bench.py --no-cpu-baseline > $E/bench_under_rocprof.json 2> $E/bench_under_rocprof.err
rc=$?; echo "trace rc=$rc"; fatal $rc trace
: > $E/configs.jsonl
# each line starts on settled clocks: the full C3-schedule search of its shape first
# (C5's 64-palette search would take ~1 min: 10 warm-up steps, ~0.1 s, instead)
for cfg in "--size 1024 --K 64 --population 1" "--population 1" "" "--size 8192 --shard-of 8" "--population 64 --steps 20 --warmup 10 --no-full-search" \
           "--dpi 96 --distance 60 --no-full-search" "--dpi 150 --distance 30 --no-full-search" \
           "--dpi 300 --distance 50 --steps 10 --warmup 2 --no-full-search" \
           "--population 64 --shard-of 8 --steps 20 --warmup 5 --no-full-search" \
           "--population 8 --steps 50 --warmup 5 --no-full-search" \
           "--size 1024 --K 1024 --steps 50 --warmup 5 --no-full-search" \
           "--size 1024 --K 4096 --steps 20 --warmup 3 --no-full-search" \
           "--size 1024 --K 8192 --steps 10 --warmup 2 --no-full-search"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $cfg >> $E/configs.jsonl 2>> $E/configs.err
  rc=$?; echo "config [$cfg] rc=$rc"; fatal $rc "config $cfg"
done
timeout -k 10 200 python bench.py --no-cpu-baseline --shard-of 8 --steps 200 > $E/shard8.json 2> $E/shard8.err
rc=$?; echo "shard8 rc=$rc"; cut -c1-200 $E/shard8.json; fatal $rc shard8
timeout -k 10 200 python bench.py --no-cpu-baseline --shard-of 8 --shard-comm --steps 200 > $E/shard8_comm.json 2> $E/shard8_comm.err
rc=$?; echo "shard8 comm rc=$rc"; cut -c1-200 $E/shard8_comm.json; fatal $rc shard8_comm
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "cost|assign|build_grid|sa_step|finalize" -f csv -d $E/traffic_$c -o run -- python3 scripts/profile_eval.py --evals 3 > $E/traffic_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; fatal $rc $c
done
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "cost|assign|build_grid" -f csv -d $E/pmc$i -o run -- python3 scripts/profile_eval.py --evals 3 > $E/pmc$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; fatal $rc pmc$i
done
exit 0
