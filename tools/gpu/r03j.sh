# after the variant pruning: conv parity (h2, variants, bf16), config 1, bench
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_j
timeout -k 10 600 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_conv_variants.py tests/test_gpu_bf16.py tests/test_gpu_config1.py tests/test_gpu_models.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1
