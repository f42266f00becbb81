# banded upsample with fused GN+SiLU (us1), k_lin1x1 (qkv/proj), spread GN-prologue transform:
# parity, bench, per-position trace
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_m
timeout -k 10 600 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_models.py tests/test_gpu_bf16.py tests/test_gpu_cond_hoist.py tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --n-steps 30 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1
