# A/B of the k_conv3lg GroupNorm-prologue transform forms (TCX_TV 0 = round 2, 1 = spread, 2 = no
# transform arithmetic: diagnostic floor, wrong results), per-layer convbench, alternating; then parity
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_k
for r in 1 2; do
  for tv in 0 1 2; do
    TCX_TV=$tv H2=1 PRO=1 REPS=30 timeout -k 10 120 python3 -u tools/convbench.py > gpurun_out/${T}_tv${tv}_$r.log 2>&1 || exit 1
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_conv_variants.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --fp32-passes 0 > gpurun_out/${T}_bench_tv1.log 2>&1 && \
TCX_TV=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --fp32-passes 0 > gpurun_out/${T}_bench_tv0.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_cfg5prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --n-steps 6 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_cfg5prof.log 2>&1
