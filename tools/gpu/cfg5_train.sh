# config 5 (256^2, 64 images per GPU) bench on the current kernels + the training step benches
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_models.py -k "chunking or h256" -x -q --timeout 200 --timeout-method thread > gpurun_out/$1_h256_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --img-size 256 --batch 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$1_bench256.log 2>&1 && \
timeout -k 10 300 python -u tools/train_bench.py score vae prior > gpurun_out/$1_train_bench.log 2>&1
