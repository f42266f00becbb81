# HBM traffic of the headline sampler's kernels: separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE)
# over a short bench run (2 sampler steps, 1 pass), per the MI355X_MICROARCH.md HBM/rocprofv3 recipe.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch -o p -- python3 bench.py --n-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write -o p -- python3 bench.py --n-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_write.log 2>&1
