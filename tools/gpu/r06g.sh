# Round 6: k_lin1x1's 8-wave 192-column form (TCX_LIN_NG): 1x1 parity tests, one-lane layer traces of the
# headline with the knob on and off, headline bench A/B alternating, config 5 A/B.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_g}
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_h2.py tests/test_gpu_passes.py -k "1x1 or lin or epilogue or attention" > gpurun_out/${T}_tests.log 2>&1 || exit 1
for f in 2 1; do
  TCX_LIN_NG=$f timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof$f -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof$f.log 2>&1 || exit 1
  python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof$f -name "*.db" | head -1) gpurun_out/${T}_layers$f.txt || exit 1
  rm -rf gpurun_out/${T}_prof$f
done
for f in 2 1 2 1; do
  echo "== TCX_LIN_NG=$f" >> gpurun_out/${T}_bench.log
  TCX_LIN_NG=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-passes 0 >> gpurun_out/${T}_bench.log 2>&1 || exit 1
done
for f in 2 1; do
  echo "== TCX_LIN_NG=$f" >> gpurun_out/${T}_c5.log
  TCX_LIN_NG=$f timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1 >> gpurun_out/${T}_c5.log 2>&1 || exit 1
done
