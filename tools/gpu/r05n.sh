# Prior DDIM launch anatomy (tools/probe/skinny_probe.hip); the 2-row upsample band (TCX_UPS_ROWS=2): its
# bit-identity test, layer traces with rows 4 / 2, bench A/B alternating.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_n}
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 120 ./tools/probe/skinny_probe > gpurun_out/${T}_skinny_probe.log 2>&1 && \
timeout -k 10 300 $P tests/test_gpu_passes.py -k "upsample_band" > gpurun_out/${T}_tests.log 2>&1 && \
for f in 4 2; do
  TCX_UPS_ROWS=$f timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof$f -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof$f.log 2>&1 || exit 1
  python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof$f -name "*.db" | head -1) gpurun_out/${T}_layers$f.txt || exit 1
  rm -rf gpurun_out/${T}_prof$f
done && \
for f in 2 4 2 4; do
  echo "== TCX_UPS_ROWS=$f" >> gpurun_out/${T}_bench.log
  TCX_UPS_ROWS=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-passes 0 >> gpurun_out/${T}_bench.log 2>&1 || exit 1
done
