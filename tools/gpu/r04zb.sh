# k_conv3m without the MFMA-dependency waits (the co-run differences were the store-data hazard):
# co-run probe with k_conv3m on, its parity tests, the headline with k_conv3m off / on / off / on.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r04_m}
TCX_CONV3M=1 timeout -k 10 200 python -u tools/determinism_probe.py --corun > gpurun_out/${T}_corun.log 2>&1 && \
grep -q "^deterministic" gpurun_out/${T}_corun.log && \
TCX_CONV3M=1 timeout -k 10 200 python -u tools/determinism_probe.py > gpurun_out/${T}_det.log 2>&1 && \
grep -q "^deterministic" gpurun_out/${T}_det.log && \
TCX_CONV3M=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_conv_variants.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_b0a.log 2>&1 && \
TCX_CONV3M=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_b1a.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_b0b.log 2>&1 && \
TCX_CONV3M=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_b1b.log 2>&1
