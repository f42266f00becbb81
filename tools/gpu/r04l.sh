# Round 4: f16x3 GEMM v3 (4-stage register pipeline) + 16-column h2_cols: tests, prior step with x3 on.
cd /root/repo
export TMPDIR=/tmp
T=r04_z
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_gemm_x3.py > gpurun_out/${T}_x3.log 2>&1 && \
TCX_PRIOR_TRAIN_X3=1 STEPS=10 WARM=3 timeout -k 10 200 python -u tools/train_bench.py prior > gpurun_out/${T}_prior.log 2>&1 && \
TCX_PRIOR_TRAIN_X3=1 STEPS=3 WARM=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_priorprof -o run -- python3 tools/train_bench.py prior > gpurun_out/${T}_priorprof.log 2>&1
