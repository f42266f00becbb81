# concurrent sampling lanes: parity test, then bench A/B over TCX_LANES = 1, 2, 3
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_models.py -k "lanes or sde" > gpurun_out/$1_tests.log 2>&1 && \
TCX_LANES=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$1_bench_l1.log 2>&1 && \
TCX_LANES=2 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$1_bench_l2.log 2>&1 && \
TCX_LANES=3 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$1_bench_l3.log 2>&1 && \
TCX_LANES=2 timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/$1_bench256_l2.log 2>&1
