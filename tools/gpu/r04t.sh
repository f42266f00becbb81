# Round 4: DDIM batch probe (skinny GEMM launch cost vs rows) + its kernel trace.
cd /root/repo
export TMPDIR=/tmp
T=r04_zd
timeout -k 10 200 python -u tools/ddim_batch_probe.py > gpurun_out/${T}_ddimB.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_ddimBprof -o run -- python3 tools/ddim_batch_probe.py > gpurun_out/${T}_ddimBprof.log 2>&1
