# Round 6: the skinny split-K reduce + LayerNorm (k_sk_reduce_ln) with its bias / residual rows in the first
# round trip and the partial planes loaded 8 at a time before their adds (same order of adds).  Prior tests on the
# new library, DDIM-50 samples of old and new compared bit for bit, three alternating pairs of DDIM-50 timing.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_ac}
LIB=vae-diffusion-toy-crystals_amd/toycrystals_amd/libtcx.so
cp $LIB abtmp/libtcx_new.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_prior.py \
  > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -3 gpurun_out/${T}_tests.txt
for v in old new; do
  cp abtmp/libtcx_$v.so $LIB
  timeout -k 10 120 python -u tools/ddim_dump.py /tmp/z_$v.npy >> gpurun_out/${T}_ab.txt 2>&1 || { cp abtmp/libtcx_new.so $LIB; exit 1; }
done
python -c "import numpy as np; a=np.load('/tmp/z_old.npy'); b=np.load('/tmp/z_new.npy'); print('DDIM-50 old vs new bit-identical:', np.array_equal(a,b), float(np.abs(a-b).max()))" >> gpurun_out/${T}_ab.txt
for rep in 1 2 3; do
  for v in old new; do
    cp abtmp/libtcx_$v.so $LIB
    echo "$v $(timeout -k 10 120 python -u tools/train_bench.py ddim 2>/dev/null | tail -1)" >> gpurun_out/${T}_ab.txt || { cp abtmp/libtcx_new.so $LIB; exit 1; }
  done
done
cp abtmp/libtcx_new.so $LIB
cat gpurun_out/${T}_ab.txt
