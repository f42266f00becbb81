# k_conv3m's GroupNorm-prologue form (PRO 1): parity, co-run determinism, the layer trace, and the
# headline A/B against the k_conv3lg / k_conv3g prologue convs (TCX_CONV3MG=0), alternating.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_b}
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 300 $P tests/test_gpu_h2.py -k "prologue or 16x16" > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 300 $P tests/test_gpu_headline.py -k "corun" >> gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 600 $P tests/test_gpu_models.py -k "forward or trained_sde300 or lanes" >> gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof -name "*.db" | head -1) gpurun_out/${T}_layers.txt && \
for v in 1 0 1 0; do
  echo "== TCX_CONV3MG=$v" >> gpurun_out/${T}_bench.log
  TCX_CONV3MG=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-passes 0 >> gpurun_out/${T}_bench.log 2>&1 || exit 1
done
