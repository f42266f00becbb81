# upsample forms A/B (TCX_UPB 0 g8, 1 band quads, 2 band groups, 3 4-row band groups), alternating
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_n
for r in 1 2; do
  for v in 0 1 2 3; do
    TCX_UPB=$v timeout -k 10 120 python3 -u tools/upbench.py >> gpurun_out/${T}_upbench.log 2>&1 || exit 1
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py -x -q -k upsample --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
