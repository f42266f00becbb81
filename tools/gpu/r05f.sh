# k_conv3m prologue-form transform schedules (tools/build_variant.sh -DTCX_M_SCHED=1/2 vs the product's
# 0): per-layer A/B, alternating, on one box; then parity of the product build.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_f}
LIB=vae-diffusion-toy-crystals_amd/toycrystals_amd/libtcx.so
cp $LIB abtmp/libtcx_s0.so
for v in s0 s1 s2 s0 s1 s2; do
  cp abtmp/libtcx_$v.so $LIB
  echo "== $v PRO=1" >> gpurun_out/${T}_conv.log
  H2=1 PRO=1 timeout -k 10 120 python -u tools/convbench.py >> gpurun_out/${T}_conv.log 2>&1 || { cp abtmp/libtcx_s0.so $LIB; exit 1; }
done
echo "== s0 PRO=0" >> gpurun_out/${T}_conv.log
cp abtmp/libtcx_s0.so $LIB
H2=1 PRO=0 timeout -k 10 120 python -u tools/convbench.py >> gpurun_out/${T}_conv.log 2>&1
