# 8-lanes-per-pixel head / first conv, paired-lane h2 upsample stores: parity tests + A/B bench + profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_models.py tests/test_gpu_h2.py > gpurun_out/$1_tests.log 2>&1 && \
TCX_PIX8=0 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --lanes-alt 0 > gpurun_out/$1_bench_off.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --lanes-alt 0 > gpurun_out/$1_bench_on.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_prof -o run -- python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes-alt 0 > gpurun_out/$1_prof.log 2>&1
