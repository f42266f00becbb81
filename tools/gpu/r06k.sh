# Round 6: the one-channel convs (thin.hip) -- their tests, the conv / wgrad / training suites they now
# serve, then the score training step with and without them (TCX_THIN=0) and its kernel breakdown.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_k}
P="python -u -m pytest -x -v -s --timeout 600 --timeout-method thread"
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "STOP rc=$rc: $*" >> gpurun_out/${T}_stop.log; exit $rc; fi; return 0; }
step timeout -k 10 600 $P tests/test_gpu_thin.py tests/test_gpu_dgrad_h2.py > gpurun_out/${T}_t1.log 2>&1
step timeout -k 10 900 $P tests/test_gpu_ops.py tests/test_gpu_wgrad.py tests/test_gpu_train.py tests/test_gpu_config1.py > gpurun_out/${T}_t2.log 2>&1
for v in "TCX_THIN=1" "TCX_THIN=0" "TCX_THIN=1" "TCX_THIN=0"; do
  echo "== $v" >> gpurun_out/${T}_train.log
  env $v STEPS=10 WARM=3 timeout -k 10 300 python -u tools/train_bench.py score vae >> gpurun_out/${T}_train.log 2>&1 || exit 1
done
STEPS=5 WARM=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 tools/train_bench.py score > gpurun_out/${T}_prof.log 2>&1 || exit 1
