# Diagnostic PMC passes on one conv layer (memory pipeline: TA/TD/L1/L2) + per-layer timing with and
# without the GroupNorm-partials epilogue.  usage: bash tools/gpu/pmc_diag.sh TAG LAYER
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1; export LAYER=$2; export H2=1 REPS=5
rocprofv3 -L > gpurun_out/${T}_counters.txt 2>&1 || true
timeout -k 10 120 python3 tools/convbench.py > gpurun_out/${T}_gn1.log 2>&1 && \
GN=0 timeout -k 10 120 python3 tools/convbench.py > gpurun_out/${T}_gn0.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcT -o p -- python3 tools/convone.py > gpurun_out/${T}_pmcT.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcA -o p -- python3 tools/convone.py > gpurun_out/${T}_pmcA.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmcL2 -o p -- python3 tools/convone.py > gpurun_out/${T}_pmcL2.log 2>&1
