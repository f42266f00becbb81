# Round 4: config 5 (256^2, bf16) bench line + one-lane kernel trace + layer timeline.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r04_cfg5
timeout -k 10 400 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 0 --no-cpu-baseline --lanes 1 --fp32-passes 0 --n-steps 20 > gpurun_out/${T}_prof.log 2>&1
