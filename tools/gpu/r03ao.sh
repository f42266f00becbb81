# training steps at the final HEAD: score x3, VAE, prior, DDIM; training kernel stats
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_ao
for r in 1 2 3; do
  STEPS=10 timeout -k 10 200 python -u tools/train_bench.py score >> gpurun_out/${T}_train.log 2>&1 || exit 1
done && \
STEPS=10 timeout -k 10 300 python -u tools/train_bench.py vae prior ddim >> gpurun_out/${T}_train.log 2>&1 && \
STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trainprof -o run -- python3 tools/train_bench.py score > gpurun_out/${T}_trainprof.log 2>&1
