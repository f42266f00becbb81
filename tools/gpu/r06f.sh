# Round 6: the whole GPU suite, config 5 A/B of up2.net.3's b2 output, and the prior step's per-process
# spread (three processes under a kernel trace: which kernels differ between a fast and a slow process).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_f}
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "STOP rc=$rc: $*" >> gpurun_out/${T}_stop.log; exit $rc; fi; return 0; }
step timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
for v in "TCX_UP21_B2=1" "TCX_UP21_B2=0" "TCX_UP21_B2=1" "TCX_UP21_B2=0"; do
  echo "== $v" >> gpurun_out/${T}_c5.log
  env $v timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1 >> gpurun_out/${T}_c5.log 2>&1 || exit 1
done
for i in 1 2 3 4; do
  STEPS=20 WARM=5 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${T}_prior$i -o run -- python3 tools/train_bench.py prior > gpurun_out/${T}_prior$i.log 2>&1 || exit 1
done
