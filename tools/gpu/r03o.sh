# slim bf16 k_conv3g at 256-px rows (config 5), band upsample fused vs apply pass, parity + benches
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_o
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_h2.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --fp32-passes 0 --lanes 1 > gpurun_out/${T}_bench_upf1_$r.log 2>&1 || exit 1
  TCX_UPF=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --fp32-passes 0 --lanes 1 > gpurun_out/${T}_bench_upf0_$r.log 2>&1 || exit 1
done && \
timeout -k 10 400 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_cfg5_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_cfg5prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --n-steps 6 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_cfg5prof.log 2>&1
