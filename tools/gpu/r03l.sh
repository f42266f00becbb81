# k_conv3lg GroupNorm-prologue schedule A/B (TCX_PRO_SCHED 0: transform over taps 5-8 / 6-8; 1: taps
# 5-6 / 6-7, tap 8 prefetches A0), per-layer convbench alternating, parity of both, one-lane benches
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_l
for r in 1 2; do
  for sc in 0 1; do
    TCX_PRO_SCHED=$sc H2=1 PRO=1 REPS=30 timeout -k 10 120 python3 -u tools/convbench.py > gpurun_out/${T}_s${sc}_$r.log 2>&1 || exit 1
  done
done
TCX_PRO_SCHED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests_s1.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests_s0.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --fp32-passes 0 > gpurun_out/${T}_bench_s0_$r.log 2>&1 || exit 1
  TCX_PRO_SCHED=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --fp32-passes 0 > gpurun_out/${T}_bench_s1_$r.log 2>&1 || exit 1
done
