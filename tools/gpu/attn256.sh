# 256x256 support: key-tiled attention + 256^2 U-Net goldens, then the whole GPU suite.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_ops.py tests/test_gpu_h2.py -k attention > gpurun_out/$1_attn.log 2>&1 && \
timeout -k 10 400 $T tests/test_gpu_models.py -k h256 > gpurun_out/$1_h256.log 2>&1 && \
timeout -k 10 900 $T tests -m gpu > gpurun_out/$1_all.log 2>&1
