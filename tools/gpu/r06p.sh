# Round 6: the halo weight gradient's ring: six stages / one workgroup per CU (TCX_W3_NS=6) vs three stages / two
# workgroups (default) at 32-pixel chunks -- tests under both, then the score step alternating.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_p}
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
TCX_W3_NS=6 timeout -k 10 300 $P tests/test_gpu_wgrad.py > gpurun_out/${T}_t1.log 2>&1 || exit 1
timeout -k 10 300 $P tests/test_gpu_wgrad.py tests/test_gpu_train.py >> gpurun_out/${T}_t1.log 2>&1 || exit 1
for v in "TCX_W3_NS=6" "TCX_W3_NS=3" "TCX_W3_NS=6" "TCX_W3_NS=3"; do
  echo "== $v" >> gpurun_out/${T}_train.log
  env $v STEPS=10 WARM=3 timeout -k 10 300 python -u tools/train_bench.py score >> gpurun_out/${T}_train.log 2>&1 || exit 1
done
TCX_W3_NS=6 STEPS=5 WARM=2 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python3 tools/train_bench.py score > gpurun_out/${T}_prof.log 2>&1 || exit 1
