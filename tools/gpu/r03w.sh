# k_head8 with hardware exp2/rcp SiLU and b128 weight reads (was 139 us avg in r03_r); config 5 k_conv3g 256-px 4 vs 8 waves
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_w
timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests_models.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 0 --lanes 1 --fp32-passes 0 --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1 && \
TCX_G256NW=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests_nw8.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline > gpurun_out/${T}_nw4_$r.log 2>&1 || exit 1
  TCX_G256NW=8 timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline > gpurun_out/${T}_nw8_$r.log 2>&1 || exit 1
done
