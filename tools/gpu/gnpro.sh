# A/B: GroupNorm+SiLU prologue (default) vs every norm as an h2 apply pass + LDS-DMA h2 conv; variant tests
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
P="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 400 $P tests/test_gpu_conv_variants.py -k "env0 or env1 or env2" > gpurun_out/${T}_variant.log 2>&1 && \
TCX_GN_PRO=0 timeout -k 10 300 $P tests/test_gpu_models.py -k "unet or sde or trained" > gpurun_out/${T}_models_nopro.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench_pro.log 2>&1 && \
TCX_GN_PRO=0 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench_nopro.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench_pro2.log 2>&1 && \
TCX_GN_PRO=0 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench_nopro2.log 2>&1
