# Round 6: config 5's b2 attention on 4 waves x 64-key tiles (three workgroups per CU): bf16 suite, config 5
# A/B alternating (TCX_ATTN_Q4), one-lane config-5 layer trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_h}
timeout -k 10 900 python -u -m pytest tests/test_gpu_bf16.py -v -s --timeout 600 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit 1
for f in 1 0 1 0; do
  echo "== TCX_ATTN_Q4=$f" >> gpurun_out/${T}_c5.log
  TCX_ATTN_Q4=$f timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1 >> gpurun_out/${T}_c5.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 0 --lanes 1 --n-steps 12 > gpurun_out/${T}_prof.log 2>&1 || exit 1
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof -name "*.db" | head -1) gpurun_out/${T}_cfg5_layers.txt
rm -rf gpurun_out/${T}_prof
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/${T}_counters.txt 2>&1 || true
