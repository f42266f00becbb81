# k_conv3m prologue form with the transform's LDS traffic as inline asm (no compiler vmcnt(0) before it)
# and the halo DMA offsets recomputed per issue (no spills): parity, co-run, per-layer, headline.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_d}
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 300 $P tests/test_gpu_h2.py -k "prologue or 16x16" > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 300 $P tests/test_gpu_headline.py -k "corun" >> gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 600 $P tests/test_gpu_models.py -k "forward or trained_sde300" >> gpurun_out/${T}_tests.log 2>&1 && \
for v in 1 0; do
  echo "== PRO=$v" >> gpurun_out/${T}_conv.log
  H2=1 PRO=$v timeout -k 10 120 python -u tools/convbench.py >> gpurun_out/${T}_conv.log 2>&1 || exit 1
done && \
for v in 1 0 1 0; do
  echo "== TCX_CONV3MG=$v" >> gpurun_out/${T}_bench.log
  TCX_CONV3MG=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-passes 0 >> gpurun_out/${T}_bench.log 2>&1 || exit 1
done
