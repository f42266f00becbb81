# config 5 (256x256, 64 images per GPU): bench line + kernel profile on the current tree
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --img-size 256 --batch 64 --steps 2 --warmup 1 --no-cpu-baseline --lanes-alt 0 > gpurun_out/$1_bench256.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_prof256 -o run -- python -u bench.py --img-size 256 --batch 64 --steps 1 --warmup 1 --no-cpu-baseline --lanes-alt 0 > gpurun_out/$1_prof256.log 2>&1
