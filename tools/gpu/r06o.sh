# Round 6: the row-striding one-channel forward kernels (thin.hip) -- their tests and the training suites
# first, then the final part B profiles (tools/gpu/r06finb.sh).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_thin.py tests/test_gpu_train.py tests/test_gpu_config1.py tests/test_gpu_ops.py > gpurun_out/r06_o_tests.log 2>&1 && \
bash tools/gpu/r06finb.sh r06_fin
