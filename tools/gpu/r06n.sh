# Round 6: the halo weight gradient with 32-pixel chunks (TCX_W3_CP=32, two workgroups per CU) vs 64-pixel
# chunks (the default): its tests under both, then the score step alternating, then the kernel trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_n}
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
TCX_W3_CP=32 timeout -k 10 300 $P tests/test_gpu_wgrad.py > gpurun_out/${T}_t1.log 2>&1 || exit 1
timeout -k 10 300 $P tests/test_gpu_wgrad.py >> gpurun_out/${T}_t1.log 2>&1 || exit 1
TCX_W3_CP=32 timeout -k 10 600 $P tests/test_gpu_train.py tests/test_gpu_config1.py > gpurun_out/${T}_t2.log 2>&1 || exit 1
for v in "TCX_W3_CP=32" "TCX_W3_CP=64" "TCX_W3_CP=32" "TCX_W3_CP=64"; do
  echo "== $v" >> gpurun_out/${T}_train.log
  env $v STEPS=10 WARM=3 timeout -k 10 300 python -u tools/train_bench.py score >> gpurun_out/${T}_train.log 2>&1 || exit 1
done
TCX_W3_CP=32 STEPS=5 WARM=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 tools/train_bench.py score > gpurun_out/${T}_prof.log 2>&1 || exit 1
