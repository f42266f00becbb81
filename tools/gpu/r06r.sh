# Round 6: the DDIM trunk's fc1 as the split-K wide skinny form with its reduce fused into the last-arriving
# workgroup (TCX_SKINNY_FC1W, default on) -- the prior tests, then the DDIM-50 call alternating on / off.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_r}
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_prior.py tests/test_gpu_models.py > gpurun_out/${T}_t1.log 2>&1 || exit 1
for v in "TCX_SKINNY_FC1W=1" "TCX_SKINNY_FC1W=0" "TCX_SKINNY_FC1W=1" "TCX_SKINNY_FC1W=0"; do
  echo "== $v" >> gpurun_out/${T}_ddim.log
  env $v STEPS=10 WARM=3 timeout -k 10 300 python -u tools/train_bench.py ddim >> gpurun_out/${T}_ddim.log 2>&1 || exit 1
done
STEPS=3 WARM=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python3 tools/train_bench.py ddim > gpurun_out/${T}_prof.log 2>&1 || exit 1
