# skinny-linear variants (TCX_SK_VAR) at the DDIM shapes, weights L2- / MALL- / HBM-resident
set -o pipefail
cd /root/repo
T=$1
for c in 1 8 24; do for v in 1 5 7 11; do SK_COPIES=$c TCX_SK_VAR=$v timeout -k 10 60 python -u tools/skbench.py >> gpurun_out/${T}_skbench.log 2>&1 || exit 1; done; done
