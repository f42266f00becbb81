# k_conv3g vs k_conv3p per U-Net layer (Bt = 256), with and without the GN prologue, and PMC passes
# of k_conv3g on up1_1 (prologue) and down2_1.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
export H2=1 REPS=20
timeout -k 10 200 env TCX_CONV3G=0 PRO=0 python3 -u tools/convbench.py > gpurun_out/${T}_conv3p.txt 2>&1 && \
timeout -k 10 200 env PRO=0 python3 -u tools/convbench.py > gpurun_out/${T}_conv3g.txt 2>&1 && \
timeout -k 10 200 env PRO=1 python3 -u tools/convbench.py > gpurun_out/${T}_conv3g_pro.txt 2>&1 && \
export REPS=5 && for L in up1_1 down2_1; do
  for PR in 0 1; do
    export LAYER=$L PRO=$PR
    timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcA_${L}_$PR -o p -- python3 tools/convbench.py > gpurun_out/${T}_pmcA_${L}_$PR.log 2>&1 || exit 1
    timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcB_${L}_$PR -o p -- python3 tools/convbench.py > gpurun_out/${T}_pmcB_${L}_$PR.log 2>&1 || exit 1
  done
done
