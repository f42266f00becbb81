# round-3 verification at HEAD: full GPU suite, smoke, default bench (4 lanes, CPU baseline, fp32 pass), one-lane rocprof stats, config 5, training steps
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_ah
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1 && \
timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5.log 2>&1 && \
STEPS=10 timeout -k 10 300 python -u tools/train_bench.py score vae prior > gpurun_out/${T}_train.log 2>&1
