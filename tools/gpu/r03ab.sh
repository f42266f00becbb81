# k_wgrad_h2 round-3 form (16-B pieces, ds_read_b64_tr_b16 operands) vs the round-2 quad-staged form (TCX_WG_R2=1):
# kernel parity, training parity, score training step A/B, kernel stats; headline + config 5 after the acf chunk change
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_tests_wgrad.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
for r in 1 2; do
  STEPS=10 timeout -k 10 200 python -u tools/train_bench.py score >> gpurun_out/${T}_train_new.log 2>&1 || exit 1
  TCX_WG_R2=1 STEPS=10 timeout -k 10 200 python -u tools/train_bench.py score >> gpurun_out/${T}_train_r2.log 2>&1 || exit 1
done && \
STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trainprof -o run -- python3 tools/train_bench.py score > gpurun_out/${T}_trainprof.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --fp32-passes 0 --lanes 1 > gpurun_out/${T}_bench1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline > gpurun_out/${T}_c5.log 2>&1
