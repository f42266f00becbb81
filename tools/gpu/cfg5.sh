# config 5 (256x256, 64 images per GPU = 512 over 8): chunking test, bench line, kernel profile.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_models.py -k "chunking or h256" > gpurun_out/$1_chunk.log 2>&1 && \
timeout -k 10 400 python -u bench.py --img-size 256 --batch 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$1_bench256.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_prof256 -o run -- python -u bench.py --img-size 256 --batch 64 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/$1_prof256.log 2>&1
