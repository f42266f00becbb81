# PRO-1 GroupNorm tables: scalar loads per chunk (TCX_TABL=0) vs LDS-staged ds_read (1), convbench alternating + parity
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_t
for r in 1 2 3; do
  for v in 0 1; do
    TCX_TABL=$v H2=1 PRO=1 REPS=30 timeout -k 10 120 python3 -u tools/convbench.py > gpurun_out/${T}_t${v}_$r.log 2>&1 || exit 1
  done
done
TCX_TABL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py -x -q -k prologue --timeout 200 --timeout-method thread > gpurun_out/${T}_tests_t1.log 2>&1
