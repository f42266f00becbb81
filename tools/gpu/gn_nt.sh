set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TCX_GN_NT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_nt -o run -- python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes-alt 0 > gpurun_out/$1_nt.log 2>&1 && \
TCX_GN_NT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1_t -o run -- python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes-alt 0 > gpurun_out/$1_t.log 2>&1
