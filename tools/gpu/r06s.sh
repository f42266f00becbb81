# Round 6 closing check on the final build: the whole GPU suite, smoke, the default bench line (with the CPU
# baseline), config 5's line and the training steps.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_s}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${T}_c5.log 2>&1 && \
STEPS=10 WARM=3 timeout -k 10 300 python -u tools/train_bench.py score vae prior ddim > gpurun_out/${T}_train.log 2>&1
