# round 4: PMC of the Winograd pair (sequential variant) beside the direct pair
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export NIC_LIB=$PWD/ab/libnic_il0.so
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" bash tools/pmc.sh r4d || exit $?
NIC_K3P=d PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" bash tools/pmc.sh r4d_direct || exit $?
python3 tools/pmc_summary.py gpurun_out/r4d_pmc > gpurun_out/r4d_summary.json 2>&1
python3 tools/pmc_summary.py gpurun_out/r4d_direct_pmc > gpurun_out/r4d_direct_summary.json 2>&1
echo done
