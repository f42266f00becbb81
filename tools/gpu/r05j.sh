# Attention kernel single-stage form (N = 256), k_attn_prep, k_head8r lookahead: the attention / passes tests,
# the headline lane identity; per-layer convs base vs a diagnostic ds build that reads its halo as if the
# source were chunk-major (TCX_DS_CM: wrong results, the refetch hypothesis); a one-lane layer trace; bench
# A/B TCX_ATTN_PREP=1/0 alternating.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_j}
LIB=vae-diffusion-toy-crystals_amd/toycrystals_amd/libtcx.so
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_passes.py tests/test_gpu_h2.py tests/test_gpu_bf16.py tests/test_gpu_headline.py -k "attention or four_lanes" > gpurun_out/${T}_tests.log 2>&1 && \
cp $LIB abtmp/libtcx_base.so && \
for v in base dscm base dscm; do
  cp abtmp/libtcx_$v.so $LIB
  echo "== $v" >> gpurun_out/${T}_conv.log
  H2=1 PRO=0 timeout -k 10 120 python -u tools/convbench.py >> gpurun_out/${T}_conv.log 2>&1 || { cp abtmp/libtcx_base.so $LIB; exit 1; }
done && \
cp abtmp/libtcx_base.so $LIB && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1 && \
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof -name "*.db" | head -1) gpurun_out/${T}_layers.txt && \
rm -rf gpurun_out/${T}_prof && \
for f in 1 0 1 0; do
  echo "== TCX_ATTN_PREP=$f" >> gpurun_out/${T}_bench.log
  TCX_ATTN_PREP=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-passes 0 >> gpurun_out/${T}_bench.log 2>&1 || exit 1
done
