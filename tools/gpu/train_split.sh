set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_train.py tests/test_gpu_scripts.py > gpurun_out/$1_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/train_bench.py score vae prior > gpurun_out/$1_bench.log 2>&1
