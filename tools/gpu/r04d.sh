# Round 4: k_conv3m timelines (in-kernel stamps) per layer shape.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r04_d
for l in down1_1 up1_0 up2_0 mid_0; do
  timeout -k 10 120 python -u tools/conv3m_stamps.py --layer $l --out gpurun_out/${T}_stamps_$l.txt > gpurun_out/${T}_stamps_$l.log 2>&1 || exit 1
done
