# DDIM-50 (native prior sampler) timing + kernel trace
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
STEPS=5 WARM=2 timeout -k 10 100 python -u tools/train_bench.py ddim > gpurun_out/${T}_ddim.log 2>&1 && \
STEPS=2 WARM=1 timeout -k 10 100 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_dprof -o run -- python -u tools/train_bench.py ddim > gpurun_out/${T}_dprof.log 2>&1
