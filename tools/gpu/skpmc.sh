# PMC passes over the skinny-linear microbenchmark (one counter group per rocprofv3 run)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "FETCH_SIZE TCC_HIT_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_BUSY_max" "TCC_EA0_RDREQ_sum TCC_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "k_skinny|k_gemm|k_conv" -d gpurun_out/${T}_pmc$i -o run --output-format csv -- python3 tools/skbench.py > gpurun_out/${T}_pmc$i.log 2>&1 || exit 1
done
