# bf16 single-product path: kernel tests, the f16x3/fp32 suites it touches, config-5 bench in bf16 and f16x3
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 300 $P tests/test_gpu_bf16.py > gpurun_out/${T}_bf16_tests.log 2>&1 && \
timeout -k 10 600 $P tests/test_gpu_h2.py tests/test_gpu_models.py -k "unet or h2 or conv or attention or sde_256" > gpurun_out/${T}_h2_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --img-size 256 --batch 64 --steps 1 --warmup 1 --no-cpu-baseline --fp32-passes 0 --precision bf16 > gpurun_out/${T}_cfg5_bf16.log 2>&1 && \
timeout -k 10 400 python -u bench.py --img-size 256 --batch 64 --steps 1 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_cfg5_f16x3.log 2>&1
