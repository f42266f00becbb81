# Round 4: x3 GEMM at occupancy 1 (4-stage pipeline without spills): tests + prior step A/B + profile.
cd /root/repo
export TMPDIR=/tmp
T=r04_zb
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm_x3.py "tests/test_gpu_train.py::test_prior_training_step_vs_reference" "tests/test_gpu_train.py::test_prior_training_step_w1024_vs_reference" > gpurun_out/${T}_tests.log 2>&1 && \
TCX_PRIOR_TRAIN_X3=1 STEPS=10 WARM=3 timeout -k 10 200 python -u tools/train_bench.py prior > gpurun_out/${T}_prior_x3.log 2>&1 && \
TCX_PRIOR_TRAIN_X3=1 STEPS=3 WARM=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_priorprof -o run -- python3 tools/train_bench.py prior > gpurun_out/${T}_priorprof.log 2>&1
