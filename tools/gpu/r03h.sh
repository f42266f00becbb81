# A/B/C of the round-3 eval fusions, one-lane bench, alternating on one box
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_h
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 --lanes 1"
for r in 1 2 3; do
  timeout -k 10 200 $B > gpurun_out/${T}_all_$r.log 2>&1 || exit 1
  TCX_GN_FOLD=0 timeout -k 10 200 $B > gpurun_out/${T}_hoist_$r.log 2>&1 || exit 1
  TCX_GN_FOLD=0 TCX_COND_HOIST=0 timeout -k 10 200 $B > gpurun_out/${T}_old_$r.log 2>&1 || exit 1
done
