# Quad epilogue with the output form compiled in (TCX_EPI_STATIC): h2 / pass / bf16 tests, one-lane
# layer traces with the knob on and off, bench A/B alternating.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_za}
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_h2.py tests/test_gpu_passes.py tests/test_gpu_bf16.py > gpurun_out/${T}_tests.log 2>&1 && \
for f in 1 0; do
  TCX_EPI_STATIC=$f timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof$f -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof$f.log 2>&1 || exit 1
  python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof$f -name "*.db" | head -1) gpurun_out/${T}_layers$f.txt || exit 1
  rm -rf gpurun_out/${T}_prof$f
done && \
for f in 1 0 1 0; do
  echo "== TCX_EPI_STATIC=$f" >> gpurun_out/${T}_bench.log
  TCX_EPI_STATIC=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-passes 0 >> gpurun_out/${T}_bench.log 2>&1 || exit 1
done
