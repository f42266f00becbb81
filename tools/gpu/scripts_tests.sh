set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_scripts.py tests/test_gpu_train.py > gpurun_out/$1_tests.log 2>&1
