# split-K GEMMs: training parity tests + the training benches (prior, score, VAE)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_train.py > gpurun_out/$1_train_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/train_bench.py prior vae score > gpurun_out/$1_train_bench.log 2>&1 && \
STEPS=3 WARM=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_pprof -o run -- python -u tools/train_bench.py prior > gpurun_out/$1_pprof.log 2>&1
