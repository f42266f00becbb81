# k_conv3lb (bf16 LDS-DMA conv, rows of 64/128/256 px): parity, config-5 bench A/B vs k_conv3g (TCX_CONV3LB=0), per-layer trace
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_x
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline > gpurun_out/${T}_lb_$r.log 2>&1 || exit 1
  TCX_CONV3LB=0 timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline > gpurun_out/${T}_g_$r.log 2>&1 || exit 1
done && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_cfg5prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --n-steps 6 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_cfg5prof.log 2>&1
