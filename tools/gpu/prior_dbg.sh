set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest -x -v -s --timeout 60 --timeout-method thread tests/test_gpu_prior.py -k "small or forward" > gpurun_out/r02_l_tests.log 2>&1 && \
TCX_NO_SKINNY=1 timeout -k 10 120 python -u -m pytest -x -v -s --timeout 60 --timeout-method thread tests/test_gpu_prior.py -k "small or forward or stepwise_and" > gpurun_out/r02_l_tests_noskinny.log 2>&1 && \
TCX_NO_SKINNY=1 STEPS=5 WARM=2 timeout -k 10 100 python -u tools/train_bench.py ddim > gpurun_out/r02_l_ddim_noskinny.log 2>&1
