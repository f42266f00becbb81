# PRO 1 raw-halo DMA spread A/B (TCX_PQ 2 / 3 / 4 taps), per-layer convbench alternating, then parity of the picks
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_s
for r in 1 2; do
  for q in 2 3 4; do
    TCX_PQ=$q H2=1 PRO=1 REPS=30 timeout -k 10 120 python3 -u tools/convbench.py > gpurun_out/${T}_q${q}_$r.log 2>&1 || exit 1
  done
done
for q in 3 4; do
  TCX_PQ=$q timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py -x -q -k prologue --timeout 200 --timeout-method thread > gpurun_out/${T}_tests_q$q.log 2>&1 || exit 1
done
