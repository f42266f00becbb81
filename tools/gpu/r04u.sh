# Round 4: DDIM with the next layer's weights prefetched into the MALL on a side stream: tests + timing + trace.
cd /root/repo
export TMPDIR=/tmp
T=r04_ze
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_prior.py > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/ddim_batch_probe.py > gpurun_out/${T}_ddimB.log 2>&1 && \
STEPS=10 WARM=3 timeout -k 10 200 python -u tools/train_bench.py ddim > gpurun_out/${T}_ddim.log 2>&1 && \
STEPS=3 WARM=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_ddimprof -o run -- python3 tools/train_bench.py ddim > gpurun_out/${T}_ddimprof.log 2>&1
