# Round 6: the split attention's bf16 attention with key tiles loaded two tiles ahead (TCX_ATTN_PF2).  Parity tests of the
# attention and the bf16 forwards, then three alternating pairs of the config-5 attention alone (tools/attnbench.py)
# and three of the config-5 sampler end to end (one tile ahead = 0 against two = 1).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_aa}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bf16.py \
  > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -3 gpurun_out/${T}_tests.txt
for rep in 1 2 3; do
  for v in 0 1; do
    TCX_ATTN_PF2=$v timeout -k 10 120 python -u tools/attnbench.py >> gpurun_out/${T}_ab.txt 2>&1 || exit 1
  done
done
A5="--img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1"
for rep in 1 2 3; do
  for v in 0 1; do
    TCX_ATTN_PF2=$v timeout -k 10 240 python -u bench.py $A5 > /tmp/b.log 2>&1 || exit 1
    echo "cfg5 TCX_ATTN_PF2=$v $(grep -o '"value": [0-9.]*' /tmp/b.log | head -1)" >> gpurun_out/${T}_ab.txt
  done
done
cat gpurun_out/${T}_ab.txt
