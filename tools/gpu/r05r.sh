# k_conv4s2g with two row blocks per wave (RT = 2, default for config 5's b2 downsamples): the bf16 / b2 and
# h2 conv tests (RT = 2 forced for every form in a second pass), config-5 bench A/B TCX_DS_RT=2/1, a config-5
# layer trace, the headline with RT forced to 2 vs 1.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_r}
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_bf16.py -k "b2 or ds" > gpurun_out/${T}_tests.log 2>&1 && \
TCX_DS_RT=2 timeout -k 10 600 $P tests/test_gpu_h2.py -k "conv_h2_vs_oracle" >> gpurun_out/${T}_tests.log 2>&1 && \
for f in 2 1 2 1; do
  echo "== TCX_DS_RT=$f" >> gpurun_out/${T}_c5.log
  TCX_DS_RT=$f timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1 >> gpurun_out/${T}_c5.log 2>&1 || exit 1
done && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 0 --lanes 1 --n-steps 20 > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof -name "*.db" | head -1) gpurun_out/${T}_layers.txt && \
rm -rf gpurun_out/${T}_prof && \
for f in 2 1; do
  echo "== TCX_DS_RT=$f" >> gpurun_out/${T}_bench.log
  TCX_DS_RT=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-passes 0 >> gpurun_out/${T}_bench.log 2>&1 || exit 1
done
