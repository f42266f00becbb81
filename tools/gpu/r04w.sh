# Round 4: k_conv3lb4 (bf16 3x3 conv, four row blocks per wave): bf16 tests, determinism at 256^2, config-5 bench A/B.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r04_lb4
timeout -k 10 200 python -u tools/dbg_bf16.py > gpurun_out/${T}_dbg.log 2>&1 && \
timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench.log 2>&1 && \
TCX_CONV3LB4=0 timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench_off.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 0 --no-cpu-baseline --lanes 1 --fp32-passes 0 --n-steps 20 > gpurun_out/${T}_prof.log 2>&1
