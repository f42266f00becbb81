# Round 6: verify the config-5 bandwidth passes (first-conv records at 1,024-px blocks, coalesced b2 head
# loads), the k_conv3mb per-layer selection, the fused Adam host path; bench config 5 / training / headline.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_e}
P="python -u -m pytest -x -v -s --timeout 600 --timeout-method thread"
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "STOP rc=$rc: $*" >> gpurun_out/${T}_stop.log; exit $rc; fi; return 0; }
step timeout -k 10 900 $P tests/test_gpu_bf16.py > gpurun_out/${T}_t1.log 2>&1
step timeout -k 10 600 $P tests/test_gpu_train.py tests/test_gpu_dp_rccl.py -k "adam or base96 or zero or training_step" > gpurun_out/${T}_t2.log 2>&1
for v in "TCX_FR_PX=1024" "TCX_FR_PX=128" "TCX_FR_PX=1024"; do
  echo "== $v" >> gpurun_out/${T}_c5.log
  env $v timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1 >> gpurun_out/${T}_c5.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 0 --lanes 1 --n-steps 12 > gpurun_out/${T}_prof.log 2>&1 || exit 1
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof -name "*.db" | head -1) gpurun_out/${T}_cfg5_layers.txt
rm -rf gpurun_out/${T}_prof
STEPS=10 WARM=3 timeout -k 10 300 python -u tools/train_bench.py score vae prior ddim > gpurun_out/${T}_train.log 2>&1 || exit 1
for i in 1 2 3; do STEPS=30 WARM=5 timeout -k 10 120 python -u tools/train_bench.py prior >> gpurun_out/${T}_prior_runs.log 2>&1 || exit 1; done
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench.log 2>&1
