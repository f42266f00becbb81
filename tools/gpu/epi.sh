# hoisted-load conv epilogue: split-path conv parity + model goldens, stamps, per-layer A/B, bench
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
P="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $P tests/test_gpu_h2.py tests/test_gpu_ops.py > gpurun_out/${T}_h2ops.log 2>&1 && \
timeout -k 10 400 $P tests/test_gpu_models.py > gpurun_out/${T}_models.log 2>&1 && \
TCX_CONV3L_DBG=1 timeout -k 10 120 python3 tools/conv3l_stamps.py > gpurun_out/${T}_dbg1.log 2>&1 && \
H2=1 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_layers_3l.log 2>&1 && \
H2=1 TCX_CONV3L=0 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_layers_3g.log 2>&1 && \
H2=1 PRO=1 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_layers_3l_pro.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench.log 2>&1 && \
TCX_CONV3L=0 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench_3g.log 2>&1
