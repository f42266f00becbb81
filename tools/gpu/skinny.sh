# Skinny-M linears + native prior: parity (tests/test_gpu_prior.py, prior/VAE goldens, training
# linears), then DDIM-50 over the 36-sample grid (native sampler) with the skinny kernels and with
# the 128-row split-K path (TCX_NO_SKINNY=1), and a kernel trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_prior.py tests/test_gpu_models.py tests/test_gpu_train.py tests/test_gpu_dp.py -k "prior or vae or linear or gemm or skinny" > gpurun_out/${T}_tests.log 2>&1 && \
STEPS=5 WARM=2 timeout -k 10 200 python -u tools/train_bench.py ddim > gpurun_out/${T}_ddim.log 2>&1 && \
TCX_NO_SKINNY=1 STEPS=5 WARM=2 timeout -k 10 200 python -u tools/train_bench.py ddim > gpurun_out/${T}_ddim_noskinny.log 2>&1 && \
STEPS=2 WARM=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_dprof -o run -- python -u tools/train_bench.py ddim > gpurun_out/${T}_dprof.log 2>&1
