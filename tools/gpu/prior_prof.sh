# FiLM prior training step (config 4 shape): bench + per-kernel profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/train_bench.py prior > gpurun_out/$1_prior.log 2>&1 && \
STEPS=3 WARM=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_pprof -o run -- python -u tools/train_bench.py prior > gpurun_out/$1_pprof.log 2>&1
