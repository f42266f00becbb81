# persistent k_conv3lg: parity (h2 tests, variants, model goldens, sampler goldens), per-layer A/B, bench A/B
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
P="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $P tests/test_gpu_h2.py > gpurun_out/${T}_h2.log 2>&1 && \
timeout -k 10 400 $P tests/test_gpu_models.py > gpurun_out/${T}_models.log 2>&1 && \
timeout -k 10 300 $P tests/test_gpu_conv_variants.py -k "env0 or env1 or env2 or env3" > gpurun_out/${T}_variant.log 2>&1 && \
H2=1 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_layers.log 2>&1 && \
H2=1 TCX_CONV3L_PERS=0 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_layers_np.log 2>&1 && \
H2=1 PRO=1 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_layers_pro.log 2>&1 && \
H2=1 PRO=1 TCX_CONV3L_PERS=0 timeout -k 10 200 python3 tools/convbench.py > gpurun_out/${T}_layers_pro_np.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench.log 2>&1 && \
TCX_CONV3L_PERS=0 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench_np.log 2>&1
