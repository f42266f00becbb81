# Config 5 bf16 3x3 conv (k_conv3lb) with the quad epilogue (5): where its run-to-run differences fall.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r04_lbwhere}
WHERE=1 DET=3 REPS=2 TCX_LB_DIAG=5 timeout -k 10 150 python -u tools/lbbench.py >> gpurun_out/${T}.log 2>&1
