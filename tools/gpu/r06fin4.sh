# Round 6: config 5's per-pass layer trace and the DDIM kernel statistics on the final tree (attention deferred max +
# two-tile-ahead loads; the prior's regrouped reduce + LayerNorm).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_fin4}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_c5prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 0 --lanes 1 --n-steps 12 > gpurun_out/${T}_c5prof.log 2>&1 && \
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_c5prof -name "*.db" | head -1) gpurun_out/${T}_cfg5_layers.txt && \
rm -rf gpurun_out/${T}_c5prof && \
STEPS=3 WARM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_ddim -o run -- python3 tools/train_bench.py ddim > gpurun_out/${T}_ddim.log 2>&1 && \
python3 tools/rocpd_stats.py $(find gpurun_out/${T}_ddim -name "*.db" | head -1) gpurun_out/${T}_ddim_kernel_stats.csv
rm -rf gpurun_out/${T}_ddim
