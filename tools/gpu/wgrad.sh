# f16x3 weight gradient: training parity, then the score training step with and without it
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_train.py > gpurun_out/${T}_train_tests.log 2>&1 && \
STEPS=10 WARM=3 timeout -k 10 200 python -u tools/train_bench.py score > gpurun_out/${T}_score.log 2>&1 && \
TCX_WGRAD_FP32=1 STEPS=10 WARM=3 timeout -k 10 200 python -u tools/train_bench.py score > gpurun_out/${T}_score_wfp32.log 2>&1 && \
STEPS=3 WARM=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_sprof -o run -- python -u tools/train_bench.py score > gpurun_out/${T}_sprof.log 2>&1
