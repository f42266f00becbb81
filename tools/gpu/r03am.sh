# hardware-SiLU h2 GroupNorm apply + round-3 verification at HEAD: full GPU suite, smoke, per-position traces (headline, config 5), default bench, one-lane rocprof stats, config 5 bench
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_am
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_cfg5prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --n-steps 6 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_cfg5prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --n-steps 20 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_stats -o run -- python3 bench.py --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_stats.log 2>&1 && \
timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5.log 2>&1
