# k_wgrad_h2: 8-byte-store staging (default) vs the round-2 2-byte form (TCX_WG_OLD=1), score training step alternating
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_u
for r in 1 2 3; do
  STEPS=10 timeout -k 10 200 python -u tools/train_bench.py score >> gpurun_out/${T}_new.log 2>&1 || exit 1
  TCX_WG_OLD=1 STEPS=10 timeout -k 10 200 python -u tools/train_bench.py score >> gpurun_out/${T}_old.log 2>&1 || exit 1
done
STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_profnew -o run -- python3 tools/train_bench.py score > gpurun_out/${T}_profnew.log 2>&1 && \
TCX_WG_OLD=1 STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_profold -o run -- python3 tools/train_bench.py score > gpurun_out/${T}_profold.log 2>&1
