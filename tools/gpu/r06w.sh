# Round 6 housekeeping: three alternating A/B pairs on one box for the split attention's XCD-grouped workgroup
# order (TCX_ATTN_XCD), at config 5 (256^2, 4,096 tokens) and on the headline (64^2).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_w}
A5="--img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1"
AH="--steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0"
for rep in 1 2 3; do
  for v in TCX_ATTN_XCD=1 TCX_ATTN_XCD=0; do
    env $v timeout -k 10 240 python -u bench.py $A5 > /tmp/b.log 2>&1 || exit 1
    echo "cfg5 $v $(grep -o '"value": [0-9.]*' /tmp/b.log | head -1)" >> gpurun_out/${T}_ab.txt
  done
done
for rep in 1 2 3; do
  for v in TCX_ATTN_XCD=1 TCX_ATTN_XCD=0; do
    env $v timeout -k 10 240 python -u bench.py $AH > /tmp/b.log 2>&1 || exit 1
    echo "headline $v $(grep -o '"value": [0-9.]*' /tmp/b.log | head -1)" >> gpurun_out/${T}_ab.txt
  done
done
