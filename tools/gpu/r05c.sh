# A/B of k_conv3m's prologue-form build variants (tools/build_variant.sh) per layer (tools/convbench.py,
# Bt = 256): base; v1 = raw halo DMA in halves over two mids; v9 = diagnostic, no transform in the loop
# (wrong results: the schedule's cost alone); agpr0 = the h2-source form without the AGPR accumulator form
# (is mfma_agpr_form still needed after the store-data fix?) + its co-run / lanes tests.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_c}
LIB=vae-diffusion-toy-crystals_amd/toycrystals_amd/libtcx.so
cp $LIB abtmp/libtcx_base.so
for v in base v1 v9 agpr0 base v1 v9 agpr0; do
  cp abtmp/libtcx_$v.so $LIB
  echo "== $v PRO=1" >> gpurun_out/${T}_conv.log
  H2=1 PRO=1 timeout -k 10 120 python -u tools/convbench.py >> gpurun_out/${T}_conv.log 2>&1 || { cp abtmp/libtcx_base.so $LIB; exit 1; }
  echo "== $v PRO=0" >> gpurun_out/${T}_conv.log
  H2=1 PRO=0 timeout -k 10 120 python -u tools/convbench.py >> gpurun_out/${T}_conv.log 2>&1 || { cp abtmp/libtcx_base.so $LIB; exit 1; }
done
cp abtmp/libtcx_agpr0.so $LIB
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_headline.py -k "corun or four_lanes" > gpurun_out/${T}_agpr0_tests.log 2>&1
rc=$?
cp abtmp/libtcx_base.so $LIB
exit $rc
