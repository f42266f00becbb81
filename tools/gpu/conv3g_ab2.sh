# k_conv3g parity (h2 tests) then per-layer timings vs k_conv3p and PMC of up1_1 (prologue).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_h2.py tests/test_gpu_models.py > gpurun_out/${T}_h2.log 2>&1 && \
export H2=1 REPS=20 && \
timeout -k 10 200 env TCX_CONV3G=0 PRO=0 python3 -u tools/convbench.py > gpurun_out/${T}_conv3p.txt 2>&1 && \
timeout -k 10 200 env PRO=0 python3 -u tools/convbench.py > gpurun_out/${T}_conv3g.txt 2>&1 && \
timeout -k 10 200 env PRO=1 python3 -u tools/convbench.py > gpurun_out/${T}_conv3g_pro.txt 2>&1 && \
export REPS=5 LAYER=up1_1 && for PR in 0 1; do
    export PRO=$PR
    timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcA_$PR -o p -- python3 tools/convbench.py > gpurun_out/${T}_pmcA_$PR.log 2>&1 || exit 1
    timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcB_$PR -o p -- python3 tools/convbench.py > gpurun_out/${T}_pmcB_$PR.log 2>&1 || exit 1
done
