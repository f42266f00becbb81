# attention: P row sums on the MFMA through an all-ones padding row of V^T, O rescale skipped when no running max moved: attention + model tests, config 5 and headline, per-position traces (vs r03_ai)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_al
timeout -k 10 900 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_bf16.py tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --fp32-passes 0 --lanes 1 > gpurun_out/${T}_h_$r.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline > gpurun_out/${T}_c5_$r.log 2>&1 || exit 1
done && \
timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c5_lanes.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_cfg5prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --n-steps 6 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_cfg5prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --n-steps 20 --steps 1 --warmup 1 --lanes 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1
