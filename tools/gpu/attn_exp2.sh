set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_h2.py -k attention > gpurun_out/$1_tests.log 2>&1 && \
timeout -k 10 300 $T tests/test_gpu_models.py > gpurun_out/$1_models.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_prof -o run -- python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes-alt 0 > gpurun_out/$1_prof.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_prof256 -o run -- python -u bench.py --img-size 256 --batch 64 --steps 1 --warmup 1 --no-cpu-baseline --lanes-alt 0 > gpurun_out/$1_prof256.log 2>&1
