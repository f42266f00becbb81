# Store-data hazard fix (store_b128_guarded): k_conv3lb with the quad epilogue repeatable, the co-run probe
# with k_conv3m on, the bf16 / h2 / model tests, config 5 and the headline with k_conv3m off / on.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r04_haz}
timeout -k 10 150 python -u tools/lbbench.py > gpurun_out/${T}_lb.log 2>&1 && \
TCX_CONV3M=1 timeout -k 10 200 python -u tools/determinism_probe.py --corun > gpurun_out/${T}_corun_m.log 2>&1 && \
timeout -k 10 200 python -u tools/determinism_probe.py > gpurun_out/${T}_det.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_h2.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench_m0.log 2>&1 && \
TCX_CONV3M=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench_m1.log 2>&1
