# PMC passes over single conv layers (tools/convone.py): one counter group per rocprofv3 run.
# usage: bash tools/gpu/pmc_conv.sh TAG "layer1 layer2" [H2=1|0]
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1; LAYERS=$2; export H2=${3:-1}
export REPS=5
rocprofv3 -L > gpurun_out/${T}_counters.txt 2>&1 || true
for L in $LAYERS; do
  export LAYER=$L
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcA_$L -o p -- python3 tools/convone.py > gpurun_out/${T}_pmcA_$L.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcB_$L -o p -- python3 tools/convone.py > gpurun_out/${T}_pmcB_$L.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcC_$L -o p -- python3 tools/convone.py > gpurun_out/${T}_pmcC_$L.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_pmcD_$L -o p -- python3 tools/convone.py > gpurun_out/${T}_pmcD_$L.log 2>&1 || exit 1
done
