# k_conv_first_sc (scalar weights) and k_head8r's 16-B constant loads: bit-identity tests (first conv),
# attention-input and headline lane tests; a one-lane layer trace; bench A/B TCX_FIRST_REC4=1/0 alternating.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_l}
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_passes.py tests/test_gpu_headline.py -k "first_conv or attention or four_lanes" > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof -name "*.db" | head -1) gpurun_out/${T}_layers.txt && \
rm -rf gpurun_out/${T}_prof && \
for f in 1 0 1 0; do
  echo "== TCX_FIRST_REC4=$f" >> gpurun_out/${T}_bench.log
  TCX_FIRST_REC4=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-passes 0 >> gpurun_out/${T}_bench.log 2>&1 || exit 1
done
