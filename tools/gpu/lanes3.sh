# bench with the lanes-default timed region (3 lanes) and with 4 lanes
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/$1_bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --lanes 4 --no-cpu-baseline > gpurun_out/$1_bench_l4.log 2>&1 && \
timeout -k 10 300 python -u bench.py --lanes 2 --no-cpu-baseline > gpurun_out/$1_bench_l2.log 2>&1
