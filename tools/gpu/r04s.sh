# Round 4: two-stage register prefetch in k_wgrad_h2 and k_gemm (raw barriers): training tests + steps + kernel trace.
cd /root/repo
export TMPDIR=/tmp
T=r04_zc
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_train.py tests/test_gpu_h2.py tests/test_gpu_gemm_x3.py tests/test_gpu_config1.py > gpurun_out/${T}_tests.log 2>&1 && \
STEPS=10 WARM=3 timeout -k 10 300 python -u tools/train_bench.py score vae prior > gpurun_out/${T}_train.log 2>&1 && \
STEPS=2 WARM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trainprof -o run -- python3 tools/train_bench.py score prior > gpurun_out/${T}_trainprof.log 2>&1
