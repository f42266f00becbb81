# Non-temporal epilogue stores for config 5's bf16 k_conv3lb (cache policy nt / sc0 nt vs default):
# per-launch timing + repeatability at the layer shapes, then config 5, alternating libraries.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r04_nt}
L=vae-diffusion-toy-crystals_amd/toycrystals_amd/libtcx.so
for v in base nt2 nt3 base nt2; do
  cp abtmp/libtcx_$v.so $L && echo "== $v" >> gpurun_out/${T}_lb.log && \
  timeout -k 10 150 python -u tools/lbbench.py >> gpurun_out/${T}_lb.log 2>&1 || exit 1
done
for v in base nt2 base nt2; do
  cp abtmp/libtcx_$v.so $L && echo "== $v" >> gpurun_out/${T}_c5.log && \
  timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --steps 1 --warmup 1 --no-cpu-baseline >> gpurun_out/${T}_c5.log 2>&1 || exit 1
done
cp abtmp/libtcx_base.so $L
