# Sampling-lane count on the round-5 kernels: bench at --lanes 4 / 3 / 2, alternating twice.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_q}
for l in 4 3 2 4 3 2; do
  echo "== lanes $l" >> gpurun_out/${T}_bench.log
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-passes 0 --lanes $l >> gpurun_out/${T}_bench.log 2>&1 || exit 1
done
