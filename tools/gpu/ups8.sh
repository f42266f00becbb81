set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
TCX_UPS8=1 timeout -k 10 300 $T tests/test_gpu_h2.py tests/test_gpu_models.py > gpurun_out/$1_tests.log 2>&1 && \
TCX_UPS8=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_on -o run -- python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes-alt 0 > gpurun_out/$1_on.log 2>&1 && \
TCX_UPS8=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_off -o run -- python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes-alt 0 > gpurun_out/$1_off.log 2>&1
