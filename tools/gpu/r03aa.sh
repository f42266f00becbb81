# k_wgrad_h2 diagnosis: PMC passes over the score training step (one counter group per rocprofv3 run)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_aa
export STEPS=1 WARM=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcA -o p -- python3 tools/train_bench.py score > gpurun_out/${T}_pmcA.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcB -o p -- python3 tools/train_bench.py score > gpurun_out/${T}_pmcB.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcC -o p -- python3 tools/train_bench.py score > gpurun_out/${T}_pmcC.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcD -o p -- python3 tools/train_bench.py score > gpurun_out/${T}_pmcD.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcE -o p -- python3 tools/train_bench.py score > gpurun_out/${T}_pmcE.log 2>&1
