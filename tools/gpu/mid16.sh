# 16-px prologue conv: k_conv3lg (TCX_CONV3L16=2, 3 transform units) vs k_conv3g; parity child + per-layer + bench
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv_variants.py -k "env4" > gpurun_out/${T}_variant.log 2>&1 && \
for k in 1 2 1 2; do H2=1 PRO=1 LAYER=mid TCX_CONV3L16=$k timeout -k 10 120 python3 tools/convbench.py >> gpurun_out/${T}_mid_$k.log 2>&1 || exit 1; done && \
TCX_CONV3L16=2 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench1.log 2>&1
