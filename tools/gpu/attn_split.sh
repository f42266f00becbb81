# f16x3 split attention: parity tests, U-Net/sampler tests, bench A/B (TCX_ATTN_SPLIT=0 vs default) at 64^2 and 256^2
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_h2.py -k attention > gpurun_out/$1_attn.log 2>&1 && \
timeout -k 10 400 $T tests/test_gpu_models.py > gpurun_out/$1_models.log 2>&1 && \
TCX_ATTN_SPLIT=0 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$1_bench_off.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$1_bench_on.log 2>&1 && \
timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/$1_bench256_on.log 2>&1
