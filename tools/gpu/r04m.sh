# Round 4: raw barriers in the GEMM chunk loops (prefetches no longer drained by __syncthreads): tests, prior step fp32 vs x3.
cd /root/repo
export TMPDIR=/tmp
T=r04_za
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm_x3.py tests/test_gpu_ops.py tests/test_gpu_train.py tests/test_gpu_prior.py > gpurun_out/${T}_tests.log 2>&1 && \
STEPS=10 WARM=3 timeout -k 10 200 python -u tools/train_bench.py prior vae score > gpurun_out/${T}_train_fp32.log 2>&1 && \
TCX_PRIOR_TRAIN_X3=1 STEPS=10 WARM=3 timeout -k 10 200 python -u tools/train_bench.py prior > gpurun_out/${T}_prior_x3.log 2>&1 && \
TCX_PRIOR_TRAIN_X3=1 STEPS=3 WARM=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_priorprof -o run -- python3 tools/train_bench.py prior > gpurun_out/${T}_priorprof.log 2>&1
