set -o pipefail
cd /root/repo
export TMPDIR=/tmp
STEPS=3 WARM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_sprof -o run -- python -u tools/train_bench.py score > gpurun_out/$1_sprof.log 2>&1
