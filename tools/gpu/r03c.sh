# per-position kernel trace of the sampler (one lane, 30 steps), GroupNorm prologue on and off
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_c
B="python3 bench.py --steps 1 --warmup 1 --n-steps 30 --no-cpu-baseline --lanes 1 --fp32-passes 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof -o run -- $B > gpurun_out/${T}_prof.log 2>&1 && \
TCX_GN_PRO=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof0 -o run -- $B > gpurun_out/${T}_prof0.log 2>&1
