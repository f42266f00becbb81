# Verification: the whole GPU suite, the layer trace of a one-lane pass and the headline bench line.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_g}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof -name "*.db" | head -1) gpurun_out/${T}_layers.txt && \
rm -rf gpurun_out/${T}_prof && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1
