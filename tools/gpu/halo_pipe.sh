# pipelined 3x3 halo kernel (TCX_HALO_PIPE=1): parity, then one-lane bench A/B and a profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TCX_HALO_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$1_pipe_tests.log 2>&1 && \
TCX_HALO_NW=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$1_nw8_tests.log 2>&1 && \
TCX_HALO_PIPE=1 timeout -k 10 200 python -u bench.py --steps 2 --lanes 1 --no-cpu-baseline > gpurun_out/$1_pipe_bench.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 2 --lanes 1 --no-cpu-baseline > gpurun_out/$1_def_bench.log 2>&1 && \
TCX_HALO_NW=8 timeout -k 10 200 python -u bench.py --steps 2 --lanes 1 --no-cpu-baseline > gpurun_out/$1_nw8_bench.log 2>&1 && \
TCX_HALO_PIPE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_pipe_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 > gpurun_out/$1_pipe_prof.log 2>&1
