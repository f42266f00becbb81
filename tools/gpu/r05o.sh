# Prior DDIM: launch anatomy probe (tools/probe/skinny_probe.hip); the wide f16x3 skinny form
# (k_skinny_h2w, fc2 partials only): prior tests, DDIM-50 A/B TCX_SKINNY_WIDE=1/0, DDIM kernel trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_o}
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"

timeout -k 10 600 $P tests/test_gpu_prior.py > gpurun_out/${T}_tests.log 2>&1 && \
for f in 1 0 1 0; do
  echo "== TCX_SKINNY_WIDE=$f" >> gpurun_out/${T}_ddim.log
  TCX_SKINNY_WIDE=$f STEPS=10 WARM=3 timeout -k 10 300 python -u tools/train_bench.py ddim prior >> gpurun_out/${T}_ddim.log 2>&1 || exit 1
done && \
STEPS=3 WARM=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_ddimprof -o run -- python3 tools/train_bench.py ddim > gpurun_out/${T}_ddimprof.log 2>&1 && \
python3 tools/rocpd_stats.py $(find gpurun_out/${T}_ddimprof -name "*.db" | head -1) gpurun_out/${T}_ddim_kernel_stats.csv && \
rm -rf gpurun_out/${T}_ddimprof
