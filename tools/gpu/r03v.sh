# config 5 (256^2 bf16): k_conv3g slim at 256-px rows with 4 waves / 256-px tiles vs 8 waves / 512-px tiles
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_v
TCX_G256NW=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests_nw8.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline > gpurun_out/${T}_nw4_$r.log 2>&1 || exit 1
  TCX_G256NW=8 timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline > gpurun_out/${T}_nw8_$r.log 2>&1 || exit 1
done
