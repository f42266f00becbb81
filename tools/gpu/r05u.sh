# bench.py after the per-configuration traffic keys: the default line (with the CPU baseline) and config 5's line.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_u}
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${T}_c5.log 2>&1 || exit 1
# and the wide skinny form with 2 column tiles x 128-deep K slices (a TCX_SKINNY_WIDE=2 variant, removed after
# this A/B: 11.15 / 11.35 vs 11.33 / 11.30 ms, profiles/r05_u_ddim_wide_ct2nc4_ab.txt): prior tests, DDIM A/B
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
TCX_SKINNY_WIDE=2 timeout -k 10 300 $P tests/test_gpu_prior.py > gpurun_out/${T}_prior_tests.log 2>&1 && \
for f in 1 2 1 2; do
  echo "== TCX_SKINNY_WIDE=$f" >> gpurun_out/${T}_ddim.log
  TCX_SKINNY_WIDE=$f STEPS=10 WARM=3 timeout -k 10 300 python -u tools/train_bench.py ddim >> gpurun_out/${T}_ddim.log 2>&1 || exit 1
done
