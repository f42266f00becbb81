# round-3 measurement: default bench line, kernel stats, per-position trace, conv traffic, training steps
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_r
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_trace -o run -- python3 bench.py --steps 1 --warmup 1 --n-steps 30 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_trace.log 2>&1 && \
bash tools/gpu/pmc_bench_traffic.sh ${T} && \
STEPS=10 timeout -k 10 300 python -u tools/train_bench.py score vae prior > gpurun_out/${T}_train_bench.log 2>&1
