# quick perf iteration: split-path parity tests, per-layer conv bench, headline bench
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$1_tests.log 2>&1 && \
H2=1 timeout -k 10 120 python -u tools/convbench.py > gpurun_out/$1_convbench_h2.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$1_bench.log 2>&1
