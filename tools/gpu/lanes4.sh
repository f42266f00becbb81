# lane 0 on the caller's stream: lane tests, bench with 3 and 4 lanes
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
P="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 400 $P tests/test_gpu_models.py -k "lane or sde or ode" > gpurun_out/${T}_lanes.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 --lanes 4 > gpurun_out/${T}_bench4.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 --lanes 2 > gpurun_out/${T}_bench2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench3b.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 --lanes 4 > gpurun_out/${T}_bench4b.log 2>&1
