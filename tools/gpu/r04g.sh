# Round 4: the whole GPU suite after the shared-epilogue change, the bench line, a one-lane kernel trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r04_g}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1
