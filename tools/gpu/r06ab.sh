# Round 6: config 5's first conv on k_conv_first_b2w (a wave per 4-channel quad, weights as scalar operands;
# TCX_FR_WAVE).  The bf16 tests (incl. the 256^2 forward bit-identical against k_conv_first_rec), three alternating
# pairs of the config-5 sampler end to end, and a kernel trace of each form.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_ab}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bf16.py \
  > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -3 gpurun_out/${T}_tests.txt
A5="--img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1"
for rep in 1 2 3; do
  for v in 0 1; do
    TCX_FR_WAVE=$v timeout -k 10 240 python -u bench.py $A5 > /tmp/b.log 2>&1 || exit 1
    echo "cfg5 TCX_FR_WAVE=$v $(grep -o '"value": [0-9.]*' /tmp/b.log | head -1)" >> gpurun_out/${T}_ab.txt
  done
done
for v in 0 1; do
  TCX_FR_WAVE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_conv_first" -d gpurun_out/${T}_prof$v -o p -- python3 bench.py $A5 > gpurun_out/${T}_prof$v.log 2>&1 || exit 1
done
cat gpurun_out/${T}_ab.txt
