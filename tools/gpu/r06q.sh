# Round 6: the whole GPU suite, smoke and a short bench on the current build (after the wgrad3h ring refactor).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_q}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1 && \
STEPS=10 WARM=3 timeout -k 10 300 python -u tools/train_bench.py score > gpurun_out/${T}_train.log 2>&1
