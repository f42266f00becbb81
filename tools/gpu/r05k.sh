# HBM write rate of the h2-record store pattern vs contiguous 1-KB store instructions (probe), and the apply pass
# with contiguous record stores (store_rec_swapped, since removed: slower), profiles/r05_k_*.
# the apply pass with contiguous record stores (store_rec_swapped): bit-identity tests, layer trace, bench A/B TCX_REC_SWAP.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_k}
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 60 ./tools/probe/store_pattern_probe > gpurun_out/${T}_probe.log 2>&1 && \
timeout -k 10 600 $P tests/test_gpu_passes.py -k "record" > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof -name "*.db" | head -1) gpurun_out/${T}_layers.txt && \
rm -rf gpurun_out/${T}_prof && \
for f in 1 0 1 0; do
  echo "== TCX_REC_SWAP=$f" >> gpurun_out/${T}_bench.log
  TCX_REC_SWAP=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-passes 0 >> gpurun_out/${T}_bench.log 2>&1 || exit 1
done
