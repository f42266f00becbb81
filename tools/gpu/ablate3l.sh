# k_conv3l ablations at up1_1 (launch time of each TCX_CONV3L_DBG variant) + PMC of the product kernel
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
for d in 1 2 3 4 5 6; do
  TCX_CONV3L_DBG=$d timeout -k 10 120 python3 tools/conv3l_stamps.py > gpurun_out/${T}_dbg$d.log 2>&1 || exit 1
done
export LAYER=up1_1 H2=1 REPS=5
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcA -o p -- python3 tools/convone.py > gpurun_out/${T}_pmcA.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CYCLES TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcB -o p -- python3 tools/convone.py > gpurun_out/${T}_pmcB.log 2>&1
