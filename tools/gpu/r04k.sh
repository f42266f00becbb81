# Round 4: f16x3 GEMM v2 (pre-split activation operands) tests + prior training step + profile; two-chain DDIM;
# bf16 suite with the column epilogue.
cd /root/repo
export TMPDIR=/tmp
T=r04_y
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_gemm_x3.py tests/test_gpu_prior.py "tests/test_gpu_train.py::test_prior_training_step_vs_reference" "tests/test_gpu_train.py::test_prior_training_step_w1024_vs_reference" > gpurun_out/${T}_x3.log 2>&1
rc=$?
echo "x3 rc $rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
STEPS=10 WARM=3 timeout -k 10 200 python -u tools/train_bench.py prior ddim > gpurun_out/${T}_prior.log 2>&1 && \
STEPS=3 WARM=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_priorprof -o run -- python3 tools/train_bench.py prior > gpurun_out/${T}_priorprof.log 2>&1 && \
STEPS=3 WARM=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_ddimprof -o run -- python3 tools/train_bench.py ddim > gpurun_out/${T}_ddimprof.log 2>&1
rc=$?
echo "prior rc $rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 380 --timeout-method thread tests/test_gpu_bf16.py > gpurun_out/${T}_bf16.log 2>&1
