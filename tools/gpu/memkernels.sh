# memory-bound side kernels (head, first conv, upsample, conditioning): GPU tests + bench + kernel profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests -m gpu > gpurun_out/$1_gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/$1_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_prof -o run -- python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes-alt 0 > gpurun_out/$1_prof.log 2>&1
