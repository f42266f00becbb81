# Round 6 closing check after the reduce + LayerNorm change: the whole GPU suite, smoke, the training steps and DDIM.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_fin3}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -n 3 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
tail -n 2 gpurun_out/${T}_smoke.log
timeout -k 10 400 python -u tools/train_bench.py score vae prior ddim > gpurun_out/${T}_train.txt 2>&1 || exit 1
cat gpurun_out/${T}_train.txt
