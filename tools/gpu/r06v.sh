# Round 6: config 5 with k_conv3lb on every 3x3 (TCX_CONV3MB=0, the new default): the bf16 tests, the bench line,
# its HBM traffic PMC (for bench.py's constant) and the per-pass layer trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_v}
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_headline.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${T}_c5.log 2>&1 && \
bash tools/gpu/r05t.sh ${T}_c5t && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_c5prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 0 --lanes 1 --n-steps 12 > gpurun_out/${T}_c5prof.log 2>&1 && \
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_c5prof -name "*.db" | head -1) gpurun_out/${T}_cfg5_layers.txt && \
rm -rf gpurun_out/${T}_c5prof
