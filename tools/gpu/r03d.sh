# fold/hoist: bit-identity + model goldens, one-lane bench A/B (alternating), per-position trace
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_e
P="python -u -m pytest -q --timeout 300 --timeout-method thread"
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 --lanes 1"
timeout -k 10 400 $P tests/test_gpu_fold_paths.py -x > gpurun_out/${T}_fold.log 2>&1 && \
timeout -k 10 500 $P tests/test_gpu_models.py -x > gpurun_out/${T}_models.log 2>&1 && \
timeout -k 10 200 $B > gpurun_out/${T}_bench_new1.log 2>&1 && \
TCX_GN_FOLD=0 TCX_COND_HOIST=0 timeout -k 10 200 $B > gpurun_out/${T}_bench_old1.log 2>&1 && \
timeout -k 10 200 $B > gpurun_out/${T}_bench_new2.log 2>&1 && \
TCX_GN_FOLD=0 TCX_COND_HOIST=0 timeout -k 10 200 $B > gpurun_out/${T}_bench_old2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --n-steps 30 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1
