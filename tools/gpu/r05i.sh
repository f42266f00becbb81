# Round-5 bandwidth passes (k_conv_first_reg, k_upsample2x_roll, k_head8r 4-pass lookahead, k_first_acf over
# distinct images): bit-identity against the round-4 forms (TCX_PASS_FORMS=r4), the quad-vs-column epilogue
# test, the headline lane identity; a one-lane layer trace; bench A/B alternating.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_i}
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_passes.py tests/test_gpu_h2.py -k "pass_forms or quad_epilogue or attention_input" > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof -name "*.db" | head -1) gpurun_out/${T}_layers.txt && \
rm -rf gpurun_out/${T}_prof && \
for f in r5 r4 r5 r4; do
  echo "== TCX_PASS_FORMS=$f" >> gpurun_out/${T}_bench.log
  TCX_PASS_FORMS=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-passes 0 >> gpurun_out/${T}_bench.log 2>&1 || exit 1
done
