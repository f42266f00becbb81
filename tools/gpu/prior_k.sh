# prior/skinny parity, DDIM-50 timing (f16x3 and fp32 trunks) and kernel trace
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_prior.py tests/test_gpu_models.py -k "prior or skinny or vae" > gpurun_out/${T}_tests.log 2>&1 && \
STEPS=5 WARM=2 timeout -k 10 100 python -u tools/train_bench.py ddim > gpurun_out/${T}_ddim.log 2>&1 && \
TCX_PRIOR_PRECISION=fp32 STEPS=5 WARM=2 timeout -k 10 100 python -u tools/train_bench.py ddim > gpurun_out/${T}_ddim_fp32.log 2>&1 && \
STEPS=2 WARM=1 timeout -k 10 100 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_dprof -o run -- python -u tools/train_bench.py ddim > gpurun_out/${T}_dprof.log 2>&1
