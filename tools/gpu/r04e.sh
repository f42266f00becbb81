# Round 4: k_conv3m with 16-B epilogue stores: h2 conv parity, stamps, bench.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r04_e}
P="python -u -m pytest -x -q -s --timeout 300 --timeout-method thread"
timeout -k 10 300 $P tests/test_gpu_h2.py -k "conv" > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/conv3m_stamps.py --layer down1_1 --out gpurun_out/${T}_stamps_down1_1.txt > /dev/null 2>&1 && \
timeout -k 10 120 python -u tools/conv3m_stamps.py --layer up1_0 --out gpurun_out/${T}_stamps_up1_0.txt > /dev/null 2>&1 && \
timeout -k 10 400 python -u bench.py --fp32-passes 0 --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1
