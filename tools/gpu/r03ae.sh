# producer-reported absmax for the split training convs (TCX_TRAIN_AMAX A/B): training tests, score step A/B, stats
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_ae
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_dp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_train_tests.log 2>&1 && \
for r in 1 2; do
  STEPS=10 timeout -k 10 200 python -u tools/train_bench.py score >> gpurun_out/${T}_train_amax.log 2>&1 || exit 1
  TCX_TRAIN_AMAX=0 STEPS=10 timeout -k 10 200 python -u tools/train_bench.py score >> gpurun_out/${T}_train_noamax.log 2>&1 || exit 1
done && \
STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trainprof -o run -- python3 tools/train_bench.py score > gpurun_out/${T}_trainprof.log 2>&1
