# A/B of the GroupNorm apply h2 pass: pipelined (libtcx.so) vs the previous loop (libtcx_gnold.so),
# alternating one-lane headline benches + the apply kernel's trace
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
D=vae-diffusion-toy-crystals_amd/toycrystals_amd
cp $D/libtcx.so /tmp/libtcx_new.so
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-passes 0 --lanes 1"
timeout -k 10 300 $B > gpurun_out/${T}_new1.log 2>&1 && cp $D/libtcx_gnold.so $D/libtcx.so && \
timeout -k 10 300 $B > gpurun_out/${T}_old1.log 2>&1 && cp /tmp/libtcx_new.so $D/libtcx.so && \
timeout -k 10 300 $B > gpurun_out/${T}_new2.log 2>&1 && cp $D/libtcx_gnold.so $D/libtcx.so && \
timeout -k 10 300 $B > gpurun_out/${T}_old2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_profold -o run -- python3 bench.py --steps 1 --warmup 0 --n-steps 20 --no-cpu-baseline --fp32-passes 0 --lanes 1 > gpurun_out/${T}_profold.log 2>&1 && cp /tmp/libtcx_new.so $D/libtcx.so && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_profnew -o run -- python3 bench.py --steps 1 --warmup 0 --n-steps 20 --no-cpu-baseline --fp32-passes 0 --lanes 1 > gpurun_out/${T}_profnew.log 2>&1
