# 4x4/s2 halo kernel: its parity cases first, then the whole GPU suite, bench, kernel profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_h2.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$1_h2_tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$1_gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/$1_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 > gpurun_out/$1_prof.log 2>&1
