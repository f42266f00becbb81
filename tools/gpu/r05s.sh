# PMC of k_conv3m's GroupNorm-prologue form (up1_1, PRO=1) vs its h2-source form on the same layer (PRO=0),
# the counter groups of r03_an (one group per pass): VALU / MFMA instructions, MFMA busy, LDS conflicts.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r05_s
export H2=1 REPS=5 LAYER=up1_1
for P in 1 0; do
  export PRO=$P
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pro${P}_A -o p -- python3 tools/convone.py > gpurun_out/${T}_pro${P}_A.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pro${P}_B -o p -- python3 tools/convone.py > gpurun_out/${T}_pro${P}_B.log 2>&1 || exit 1
done
