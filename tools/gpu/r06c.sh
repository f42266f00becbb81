# Round 6: k_conv3mb (config 5's 3x3 convs on 16x16x32 bf16 tap pairs) — parity and repeat tests first,
# then per-layer timing against k_conv3lb (2- and 3-slot rings), then the config-5 bench A/B.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_c}
P="python -u -m pytest -x -v -s --timeout 600 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_bf16.py -k "conv3mb or b2_conv_equals or chunk_major or conv3lb_repeats" > gpurun_out/${T}_t1.log 2>&1 || exit 1
for v in "TCX_CONV3MB=2" "TCX_CONV3MB=0 TCX_LB_RING=3" "TCX_CONV3MB=0 TCX_LB_RING=2"; do
  env $v timeout -k 10 300 python -u tools/mbbench.py >> gpurun_out/${T}_layers.log 2>&1 || exit 1
done
for v in "TCX_CONV3MB=1" "TCX_CONV3MB=0" "TCX_CONV3MB=1"; do
  echo "== $v" >> gpurun_out/${T}_c5.log
  env $v timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1 >> gpurun_out/${T}_c5.log 2>&1 || exit 1
done
timeout -k 10 900 $P tests/test_gpu_bf16.py > gpurun_out/${T}_t2.log 2>&1
