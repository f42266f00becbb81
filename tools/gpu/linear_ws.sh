set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_scripts.py > gpurun_out/$1_tests.log 2>&1 && \
STEPS=5 WARM=2 timeout -k 10 200 python -u tools/train_bench.py ddim prior vae > gpurun_out/$1_bench.log 2>&1
