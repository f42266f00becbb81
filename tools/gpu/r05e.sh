# k_conv3m prologue form, one transform task per MFMA gap (value parts A / B): parity + per-layer A/B.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_e}
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 300 $P tests/test_gpu_h2.py -k "prologue or 16x16" > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 300 $P tests/test_gpu_headline.py -k "corun" >> gpurun_out/${T}_tests.log 2>&1 && \
for v in 1 0 1 0; do
  echo "== PRO=$v" >> gpurun_out/${T}_conv.log
  H2=1 PRO=$v timeout -k 10 120 python -u tools/convbench.py >> gpurun_out/${T}_conv.log 2>&1 || exit 1
done
