# k_wgrad_h2 with 8-byte LDS stores: training parity + score step timing + kernel stats
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_p
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
STEPS=10 timeout -k 10 300 python -u tools/train_bench.py score vae prior > gpurun_out/${T}_train_bench.log 2>&1 && \
STEPS=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 tools/train_bench.py score > gpurun_out/${T}_prof.log 2>&1
