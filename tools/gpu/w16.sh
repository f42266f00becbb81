# k_conv3lg at 16-px rows (mid block): parity, variant children, per-layer A/B, bench
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
P="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $P tests/test_gpu_h2.py > gpurun_out/${T}_h2.log 2>&1 && \
timeout -k 10 400 $P tests/test_gpu_models.py > gpurun_out/${T}_models.log 2>&1 && \
timeout -k 10 400 $P tests/test_gpu_conv_variants.py -k "env0 or env1 or env2 or env3 or env4" > gpurun_out/${T}_variant.log 2>&1 && \
H2=1 LAYER=mid timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_mid.log 2>&1 && \
H2=1 LAYER=mid TCX_CONV3L16=0 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_mid_3g.log 2>&1 && \
H2=1 PRO=1 LAYER=mid timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_mid_pro.log 2>&1 && \
H2=1 PRO=1 LAYER=mid TCX_CONV3L16=0 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_mid_pro_3g.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench.log 2>&1 && \
TCX_CONV3L16=0 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench_3g.log 2>&1
