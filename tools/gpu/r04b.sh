# Round 4: MFMA shape probe (32x32x16 vs 16x16x32 f16 at equal FLOPs), the config-1 teacher-forced
# gradients and the w1024 prior training step against their reference goldens.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r04_b
timeout -k 10 120 tools/probe/mfma_shape_probe 4000 > gpurun_out/${T}_mfma_shape.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_config1.py tests/test_gpu_train.py -k "teacher or w1024" > gpurun_out/${T}_tests.log 2>&1
