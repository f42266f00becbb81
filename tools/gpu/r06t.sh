# Round 6: first-conv record kernel with 4 / 2 / 1 pixels per thread item (TCX_FR_PPT; outputs bit-identical):
# the whole GPU suite and smoke with TCX_FR_PPT=4, then the kernel's duration per variant from kernel traces
# of one-lane sampling passes, then the bench line alternating 4 / 1.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_t}
TCX_FR_PPT=4 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || exit 1
TCX_FR_PPT=4 timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
for v in 4 2 1; do
  TCX_FR_PPT=$v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_p$v -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --lanes 1 --fp32-passes 0 --n-steps 20 > gpurun_out/${T}_p$v.log 2>&1 || exit 1
  python3 tools/rocpd_stats.py $(find gpurun_out/${T}_p$v -name "*.db" | head -1) > gpurun_out/${T}_p${v}_stats.csv || exit 1
  rm -rf gpurun_out/${T}_p$v
done
for v in 4 1 4 1; do
  echo "== TCX_FR_PPT=$v" >> gpurun_out/${T}_bench.log
  TCX_FR_PPT=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > /tmp/b.log 2>&1 || exit 1
  grep "^{" /tmp/b.log >> gpurun_out/${T}_bench.log
done
