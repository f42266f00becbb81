# Round 4: bf16 suite after reverting k_conv's AGPR form; prior training step + DDIM kernel traces.
cd /root/repo
export TMPDIR=/tmp
T=r04_v
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 280 --timeout-method thread tests/test_gpu_bf16.py > gpurun_out/${T}_bf16.log 2>&1
rc=$?
echo "bf16 rc $rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
STEPS=10 WARM=3 timeout -k 10 200 python -u tools/train_bench.py prior ddim > gpurun_out/${T}_prior.log 2>&1 && \
STEPS=3 WARM=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_priorprof -o run -- python3 tools/train_bench.py prior > gpurun_out/${T}_priorprof.log 2>&1 && \
STEPS=3 WARM=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_ddimprof -o run -- python3 tools/train_bench.py ddim > gpurun_out/${T}_ddimprof.log 2>&1
