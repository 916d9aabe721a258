# Two PMC passes over one kernel (default: the cost kernels; KREGEX selects another),
# profile_eval with 3 evaluations ($PROF_ARGS passed on), averaged per kernel.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "${KREGEX:-cost}" -f csv -d gpurun_out/pmc/${TAG:-x}$i -o run -- python3 scripts/profile_eval.py --evals 3 ${PROF_ARGS:-} > gpurun_out/pmc/${TAG:-x}$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -3 gpurun_out/pmc/${TAG:-x}$i.log; exit $rc; fi
done
python3 scripts/pmc_summary.py gpurun_out/pmc/${TAG:-x}1 gpurun_out/pmc/${TAG:-x}2
