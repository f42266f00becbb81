# Non-temporal epilogue stores on every split-path conv (f16x3 headline) vs bf16 only: alternating libraries.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r04_ntall}
L=vae-diffusion-toy-crystals_amd/toycrystals_amd/libtcx.so
for v in base ntall base ntall; do
  cp abtmp/libtcx_$v.so $L && echo "== $v" >> gpurun_out/${T}.log && \
  timeout -k 10 300 python -u bench.py --no-cpu-baseline >> gpurun_out/${T}.log 2>&1 || exit 1
done
cp abtmp/libtcx_base.so $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -m gpu -x -q -k repeats --timeout 200 --timeout-method thread > gpurun_out/${T}_rep.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1
