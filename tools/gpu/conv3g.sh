# k_conv3g (512-pixel 3x3 tiles + GroupNorm+SiLU prologue): its parity cases, the model goldens,
# then the headline bench and a one-lane kernel trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
P="python -u -m pytest -x -v -s --timeout 200 --timeout-method thread"
timeout -k 10 300 $P tests/test_gpu_h2.py > gpurun_out/${T}_h2.log 2>&1 && \
timeout -k 10 400 $P tests/test_gpu_models.py > gpurun_out/${T}_models.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1
