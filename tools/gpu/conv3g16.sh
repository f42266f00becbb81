# k_conv3g at 16-pixel rows (mid block, with the mid GroupNorm prologue): parity (h2, bf16, model
# tests), per-layer A/B vs k_conv3p, the headline bench, the bf16 config-5 bench and a kernel trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_h2.py tests/test_gpu_bf16.py tests/test_gpu_models.py > gpurun_out/${T}_tests.log 2>&1 && \
export H2=1 REPS=20 && \
timeout -k 10 200 env TCX_CONV3G=0 PRO=0 python3 -u tools/convbench.py > gpurun_out/${T}_conv3p.txt 2>&1 && \
timeout -k 10 200 env PRO=1 python3 -u tools/convbench.py > gpurun_out/${T}_conv3g_pro.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1
