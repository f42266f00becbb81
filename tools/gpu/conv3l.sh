# k_conv3l (B fragments staged once per workgroup in an LDS ring): parity (split-path conv cases,
# prologue cases, the k_conv3g variant child), per-layer A/B against k_conv3g, the headline bench.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
P="python -u -m pytest -x -v -s --timeout 200 --timeout-method thread"
timeout -k 10 300 $P tests/test_gpu_h2.py -k "conv" > gpurun_out/${T}_h2.log 2>&1 && \
timeout -k 10 300 $P tests/test_gpu_conv_variants.py -k "env0" > gpurun_out/${T}_variant.log 2>&1 && \
H2=1 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_layers_3l.log 2>&1 && \
H2=1 TCX_CONV3L=0 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_layers_3g.log 2>&1 && \
H2=1 PRO=1 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_layers_3l_pro.log 2>&1 && \
H2=1 PRO=1 TCX_CONV3L=0 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_layers_3g_pro.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench.log 2>&1
