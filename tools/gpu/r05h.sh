# Config 5's 2-byte bf16 tensors (b2): parity (b2 vs records bit for bit, writers, attention, the 256^2
# forward and sampler), then the config-5 bench A/B against the 4-byte records (TCX_BF_B2=0) and a layer trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_h}
P="python -u -m pytest -x -v -s --timeout 600 --timeout-method thread"
timeout -k 10 900 $P tests/test_gpu_bf16.py > gpurun_out/${T}_tests.log 2>&1 && \
for v in 1 0; do
  echo "== TCX_BF_B2=$v" >> gpurun_out/${T}_c5.log
  TCX_BF_B2=$v timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1 >> gpurun_out/${T}_c5.log 2>&1 || exit 1
done && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 0 --lanes 1 --n-steps 20 > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof -name "*.db" | head -1) gpurun_out/${T}_layers.txt && \
rm -rf gpurun_out/${T}_prof
