# Round 4: k_conv3m (16x16x32 MFMA, h2-source 3x3 convs): parity (h2 ops + model goldens), the bench
# line, and a one-lane kernel trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r04_c}
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_h2.py tests/test_gpu_models.py > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1
