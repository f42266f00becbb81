# Config 5 (256^2 bf16, b2 tensors): kernel trace of a one-lane sampling pass reported pass by pass
# (tools/rocpd_layers.py), then PMC of the 3x3 bf16 convs k_conv3lb<256> / <128> (MFMA busy,
# VALU / MFMA, LDS bank conflicts) — one counter group per pass.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_a}
A="--img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 0 --lanes 1"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python3 bench.py $A --n-steps 12 > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof -name "*.db" | head -1) gpurun_out/${T}_cfg5_layers.txt && \
rm -rf gpurun_out/${T}_prof && \
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_conv3lb" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_A -o p -- python3 bench.py $A --n-steps 2 > gpurun_out/${T}_A.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_conv3lb" --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_B -o p -- python3 bench.py $A --n-steps 2 > gpurun_out/${T}_B.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_conv3lb|k_conv4s2g|k_attention" --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_F -o p -- python3 bench.py $A --n-steps 2 > gpurun_out/${T}_F.log 2>&1 && \
for k in "k_conv3lb<256>" "k_conv3lb<128>" "k_conv3lb<64>"; do
  echo "== $k" >> gpurun_out/${T}_pmc.txt
  python3 tools/pmc_summary.py "$k" gpurun_out/${T}_A gpurun_out/${T}_B >> gpurun_out/${T}_pmc.txt || exit 1
done && \
python3 tools/pmc_summary.py "k_conv4s2g<128" gpurun_out/${T}_F >> gpurun_out/${T}_pmc.txt && \
python3 tools/pmc_summary.py "k_conv4s2g<64" gpurun_out/${T}_F >> gpurun_out/${T}_pmc.txt && \
python3 tools/pmc_summary.py "k_attention" gpurun_out/${T}_F >> gpurun_out/${T}_pmc.txt && \
tar czf gpurun_out/${T}_pmc_raw.tgz gpurun_out/${T}_A gpurun_out/${T}_B gpurun_out/${T}_F && rm -rf gpurun_out/${T}_A gpurun_out/${T}_B gpurun_out/${T}_F
