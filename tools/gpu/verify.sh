# Round verification: new parity tests first (printed values), the whole GPU suite, smoke, the
# bench line, a one-lane kernel trace, and the PMC traffic passes of the headline sampler.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_models.py -k "sampler or trained or h256" tests/test_gpu_dp.py > gpurun_out/${T}_new_tests.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch -o p -- python3 bench.py --n-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --fp32-passes 0 --lanes 1 > gpurun_out/${T}_fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write -o p -- python3 bench.py --n-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --fp32-passes 0 --lanes 1 > gpurun_out/${T}_write.log 2>&1
