# Round 4: bisect the bf16 256^2 forward (quad vs column epilogue build) + the f16x3 GEMM tests + prior step.
cd /root/repo
export TMPDIR=/tmp
T=r04_w
timeout -k 10 200 python -u tools/dbg_bf16.py > gpurun_out/${T}_dbg_quad.log 2>&1 && \
timeout -k 10 200 python -u tools/dbg_bf16.py --lib build_dbg/libtcx_cols.so > gpurun_out/${T}_dbg_cols.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_gemm_x3.py "tests/test_gpu_train.py::test_prior_training_step_vs_reference" "tests/test_gpu_train.py::test_prior_training_step_w1024_vs_reference" > gpurun_out/${T}_x3.log 2>&1
rc=$?
echo "rc $rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
STEPS=10 WARM=3 timeout -k 10 200 python -u tools/train_bench.py prior > gpurun_out/${T}_prior.log 2>&1 && \
STEPS=3 WARM=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_priorprof -o run -- python3 tools/train_bench.py prior > gpurun_out/${T}_priorprof.log 2>&1
