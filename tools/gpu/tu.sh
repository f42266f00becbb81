# prologue form of k_conv3lg with 3 transform units at 32-px rows: parity, per-layer and bench A/B vs k_conv3l
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
P="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
TCX_CONV3L_GLDS_PRO=1 timeout -k 10 300 $P tests/test_gpu_h2.py > gpurun_out/${T}_h2.log 2>&1 && \
timeout -k 10 400 $P tests/test_gpu_conv_variants.py -k "env2 or env6" > gpurun_out/${T}_variant.log 2>&1 && \
TCX_CONV3L_GLDS_PRO=1 timeout -k 10 400 $P tests/test_gpu_models.py > gpurun_out/${T}_models.log 2>&1 && \
H2=1 PRO=1 TCX_CONV3L_GLDS_PRO=1 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_layers_g.log 2>&1 && \
H2=1 PRO=1 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_layers.log 2>&1 && \
TCX_CONV3L_GLDS_PRO=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench_g.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench.log 2>&1 && \
TCX_CONV3L_GLDS_PRO=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench_g2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench2.log 2>&1
