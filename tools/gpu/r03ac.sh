# training convs with fragment-ordered weights (k_conv3lg / k_conv4s2g) vs register-staged (TCX_TRAIN_FRAG=0): full GPU suite, score step A/B, stats
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_ac
timeout -k 10 1100 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 && \
for r in 1 2; do
  STEPS=10 timeout -k 10 200 python -u tools/train_bench.py score >> gpurun_out/${T}_train_frag.log 2>&1 || exit 1
  TCX_TRAIN_FRAG=0 STEPS=10 timeout -k 10 200 python -u tools/train_bench.py score >> gpurun_out/${T}_train_nofrag.log 2>&1 || exit 1
done && \
STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trainprof -o run -- python3 tools/train_bench.py score > gpurun_out/${T}_trainprof.log 2>&1 && \
timeout -k 10 300 python -u tools/train_bench.py vae prior > gpurun_out/${T}_train_vae_prior.log 2>&1
