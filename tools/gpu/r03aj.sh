# k_first_acf with 1024-pixel chunks at 64^2: model tests, one-lane headline, per-position trace (vs r03_ai)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_aj
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_bf16.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --fp32-passes 0 --lanes 1 > gpurun_out/${T}_h_1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --n-steps 20 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1
