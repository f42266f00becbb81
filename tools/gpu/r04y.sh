# Persistent k_conv3lg (PRO 0) A/B: determinism alone and co-run, the h2 conv / model tests, bench with the
# persistent form on and off.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r04_pers}
timeout -k 10 200 python -u tools/determinism_probe.py > gpurun_out/${T}_det.log 2>&1 && \
timeout -k 10 200 python -u tools/determinism_probe.py --corun > gpurun_out/${T}_corun.log 2>&1 && \
grep -q "^deterministic" gpurun_out/${T}_det.log && grep -q "^deterministic" gpurun_out/${T}_corun.log && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_models.py tests/test_gpu_conv_variants.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
TCX_CONV3LG_PERS=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench_on.log 2>&1 && \
TCX_CONV3LG_PERS=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench_off.log 2>&1 && \
TCX_CONV3LG_PERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1
