# PMC passes on the cost/assign kernels for profile_eval configurations.
# CFGS: ';'-separated profile_eval argument sets; results in gpurun_out/pmc/c<i>/p<j>.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
stop_if_fatal() { if [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; then echo "fatal rc=$1 at $2"; exit "$1"; fi; }
IFS=';' read -r -a cfgs <<< "${CFGS:-${CFG:-}}"
ci=0
for cfg in "${cfgs[@]}"; do
ci=$((ci+1)); mkdir -p gpurun_out/pmc/c$ci
i=0
for pmc in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE" \
           "SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_INSTS_BRANCH SQ_INSTS_SALU SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAIT_INST_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU" \
           "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INST_LEVEL_VMEM SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --kernel-include-regex "cost_|assign" -f csv -d gpurun_out/pmc/c$ci/p$i -o run -- python3 scripts/profile_eval.py --evals 2 $cfg > gpurun_out/pmc/c$ci/p$i.log 2>&1
  rc=$?; echo "cfg$ci pmc$i rc=$rc"; stop_if_fatal $rc pmc$i
done
done
exit 0
