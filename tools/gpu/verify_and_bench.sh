# round-end style verification: smoke, the whole GPU suite, the default bench line, a kernel profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$1_smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$1_gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/$1_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes-alt 0 > gpurun_out/$1_prof.log 2>&1
