# 3x3 halo kernel variants: parity (h2 + model tests) and one-lane bench per variant
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TCX_HALO_NW=4 TCX_HALO_RT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$1_rt2_tests.log 2>&1 && \
TCX_HALO_NW=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$1_w_tests.log 2>&1 && \
TCX_HALO_NW=4 TCX_HALO_RT=2 timeout -k 10 200 python -u bench.py --steps 2 --lanes 1 --no-cpu-baseline > gpurun_out/$1_rt2_bench.log 2>&1 && \
TCX_HALO_NW=0 timeout -k 10 200 python -u bench.py --steps 2 --lanes 1 --no-cpu-baseline > gpurun_out/$1_w_bench.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 2 --lanes 1 --no-cpu-baseline > gpurun_out/$1_def_bench.log 2>&1 && \
TCX_HALO_NW=4 TCX_HALO_RT=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_rt2_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 > gpurun_out/$1_rt2_prof.log 2>&1
