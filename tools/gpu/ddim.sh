set -o pipefail
cd /root/repo
export TMPDIR=/tmp
STEPS=5 WARM=2 timeout -k 10 200 python -u tools/train_bench.py ddim > gpurun_out/$1_ddim.log 2>&1 && \
STEPS=2 WARM=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_dprof -o run -- python -u tools/train_bench.py ddim > gpurun_out/$1_dprof.log 2>&1
