# Round-6 final verification, part B: kernel-trace stats of the one-lane pass and its layer roofline table, HBM
# traffic PMC passes at the roofline's configuration (one lane: Bt = 256 per launch) and at config 5, config 5's
# per-pass layer trace, the training steps and the DDIM kernel trace.  Stops at the first failing step.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_fin}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof -name "*.db" | head -1) gpurun_out/${T}_layers.txt && \
python3 tools/layer_roofline.py gpurun_out/${T}_layers.txt > gpurun_out/${T}_layer_roofline.txt 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch -o p -- python3 bench.py --n-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --fp32-passes 0 --lanes 1 > gpurun_out/${T}_fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write -o p -- python3 bench.py --n-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --fp32-passes 0 --lanes 1 > gpurun_out/${T}_write.log 2>&1 && \
python3 tools/pmc_traffic.py gpurun_out/${T}_fetch gpurun_out/${T}_write > gpurun_out/${T}_pmc_traffic.txt 2>&1 && \
rm -rf gpurun_out/${T}_fetch gpurun_out/${T}_write && \
bash tools/gpu/r05t.sh ${T}_c5t && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_c5prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 0 --lanes 1 --n-steps 12 > gpurun_out/${T}_c5prof.log 2>&1 && \
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_c5prof -name "*.db" | head -1) gpurun_out/${T}_cfg5_layers.txt && \
rm -rf gpurun_out/${T}_c5prof && \
STEPS=10 WARM=3 timeout -k 10 300 python -u tools/train_bench.py score vae prior ddim > gpurun_out/${T}_train.log 2>&1 && \
STEPS=3 WARM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_ddim -o run -- python3 tools/train_bench.py ddim > gpurun_out/${T}_ddim.log 2>&1
