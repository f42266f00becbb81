# Round 4 first GPU call: bench.py's own N-rank path (2 ranks on the one GPU over gloo) and the default bench line.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r04_a
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_bench_dist.py > gpurun_out/${T}_bench_dist.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1
