# PMC of k_conv3lg at up1_1 and a one-lane kernel trace of the headline sampler
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
export LAYER=up1_1 H2=1 REPS=5
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcA -o p -- python3 tools/convone.py > gpurun_out/${T}_pmcA.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CYCLES TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcB -o p -- python3 tools/convone.py > gpurun_out/${T}_pmcB.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_LEVEL_WAVES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcC -o p -- python3 tools/convone.py > gpurun_out/${T}_pmcC.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1
