# Round 6: the halo-staged 3x3 weight gradient (wgrad3h.hip) -- its tests first (each under its own limit), then
# the training suites, then the score step with it on / off (TCX_WGRAD3H) and the kernel breakdown.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_l}
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 300 $P tests/test_gpu_wgrad.py > gpurun_out/${T}_t1.log 2>&1 || exit 1
timeout -k 10 900 $P tests/test_gpu_thin.py tests/test_gpu_dgrad_h2.py tests/test_gpu_train.py tests/test_gpu_config1.py > gpurun_out/${T}_t2.log 2>&1 || exit 1
for v in "TCX_WGRAD3H=1" "TCX_WGRAD3H=0" "TCX_WGRAD3H=1" "TCX_WGRAD3H=0"; do
  echo "== $v" >> gpurun_out/${T}_train.log
  env $v STEPS=10 WARM=3 timeout -k 10 300 python -u tools/train_bench.py score >> gpurun_out/${T}_train.log 2>&1 || exit 1
done
STEPS=5 WARM=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 tools/train_bench.py score > gpurun_out/${T}_prof.log 2>&1 || exit 1
