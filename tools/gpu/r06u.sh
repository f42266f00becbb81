# Round 6 housekeeping: three alternating A/B pairs on one box for each sub-1 % config-5 change kept this round
# -- the first-conv record kernel's 1,024-pixel workgroups at 256^2 rows (TCX_FR_PX), k_conv3lb's three-slot
# weight ring (TCX_LB_RING) and k_conv3mb on the Cin >= 192 b2-output layers (TCX_CONV3MB).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_u}
A="--img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1"
for knob in "TCX_FR_PX=1024 TCX_FR_PX=128" "TCX_LB_RING=3 TCX_LB_RING=2" "TCX_CONV3MB=1 TCX_CONV3MB=0"; do
  set -- $knob
  for rep in 1 2 3; do
    for v in "$1" "$2"; do
      env $v timeout -k 10 240 python -u bench.py $A > /tmp/b.log 2>&1 || exit 1
      echo "$v $(grep -o '"value": [0-9.]*' /tmp/b.log | head -1)" >> gpurun_out/${T}_ab.txt
    done
  done
done
