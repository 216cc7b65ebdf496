# PMC passes of the product QT kernel on C3 at 2^26 (TAG names the files) (explore.py through the
# product library), one rocprofv3 --pmc run per counter group.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
export XFG_LIB=$GRAFT_REPO_ROOT/xdp-tools_amd/lib/libxdpfilter_gpu.so KNAME=pipeq
TAG=${TAG:-r04} bash tools/pmc.sh ${TAG:-r04} "--log2-packets 26 1000000:500:250" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" \
  "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" \
  "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"
