cd /root/repo
export TMPDIR=/tmp
T=r04_v
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 280 --timeout-method thread tests/test_gpu_bf16.py > gpurun_out/${T}_bf16.log 2>&1
