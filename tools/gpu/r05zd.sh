# k_conv3m with non-temporal output stores (fp32 and paired h2): h2 / pass tests on the new library,
# one-lane layer traces of the base and new libraries,
# bench A/B alternating (libraries swapped in place).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_zd}
LIB=vae-diffusion-toy-crystals_amd/toycrystals_amd/libtcx.so
P="python -u -m pytest -x -q --timeout 400 --timeout-method thread"
cp abtmp/libtcx_new.so $LIB && \
timeout -k 10 900 $P tests/test_gpu_h2.py tests/test_gpu_passes.py > gpurun_out/${T}_tests.log 2>&1 && \
for v in new base; do
  cp abtmp/libtcx_$v.so $LIB || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof$v -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof$v.log 2>&1 || exit 1
  python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof$v -name "*.db" | head -1) gpurun_out/${T}_layers$v.txt || exit 1
  rm -rf gpurun_out/${T}_prof$v
done && \
for v in new base new base; do
  cp abtmp/libtcx_$v.so $LIB || exit 1
  echo "== $v" >> gpurun_out/${T}_bench.log
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-passes 0 >> gpurun_out/${T}_bench.log 2>&1 || exit 1
done
