# Round 6: k_gemm_reduce (split-K reduce + epilogue of the training GEMMs) with every operand requested before the first
# add (partials 8 at a time, same order).  Training / prior tests on the new library, three prior training steps of the
# old and new library compared bit for bit, three alternating pairs of the prior training step.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_ad}
LIB=vae-diffusion-toy-crystals_amd/toycrystals_amd/libtcx.so
cp $LIB abtmp/libtcx_new.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_prior.py \
  > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -n 2 gpurun_out/${T}_tests.txt
for v in old new; do
  cp abtmp/libtcx_$v.so $LIB
  timeout -k 10 180 python -u tools/prior_train_dump.py /tmp/p_$v.npz >> gpurun_out/${T}_ab.txt 2>&1 || { cp abtmp/libtcx_new.so $LIB; exit 1; }
done
python -c "
import numpy as np
a=np.load('/tmp/p_old.npz'); b=np.load('/tmp/p_new.npz')
print('prior params after 3 steps, old vs new bit-identical:', all(np.array_equal(a[k], b[k]) for k in a.files), len(a.files))" >> gpurun_out/${T}_ab.txt
for rep in 1 2 3; do
  for v in old new; do
    cp abtmp/libtcx_$v.so $LIB
    echo "$v $(timeout -k 10 180 python -u tools/train_bench.py prior 2>/dev/null | tail -1)" >> gpurun_out/${T}_ab.txt || { cp abtmp/libtcx_new.so $LIB; exit 1; }
  done
done
cp abtmp/libtcx_new.so $LIB
cat gpurun_out/${T}_ab.txt
