# Round 6 verification: new tests (b2 chunk-major skips, misaligned head weights, base-96 training golden,
# RCCL-forced DP + ZeRO-1, the DP scripts at world 2 / 3), then config 5 A/B (chunk-major skips, attention XCD
# order, conv3lb weight ring), config-5 traffic PMC and layer trace, a short headline bench.
# A test FAILURE (pytest rc 1) does not stop the script; a timeout, abort or crash (rc >= 124) does.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_b}
P="python -u -m pytest -x -v -s --timeout 600 --timeout-method thread"
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "STOP rc=$rc: $*" >> gpurun_out/${T}_stop.log; exit $rc; fi; return 0; }
step timeout -k 10 600 $P tests/test_gpu_bf16.py -k "chunk_major or misaligned" > gpurun_out/${T}_t1.log 2>&1
step timeout -k 10 600 $P tests/test_gpu_train.py -k "base96 or base32" > gpurun_out/${T}_t2.log 2>&1
step timeout -k 10 900 $P tests/test_gpu_dp_rccl.py > gpurun_out/${T}_t3.log 2>&1
for v in "TCX_SKIP_CM=3" "TCX_SKIP_CM=0" "TCX_ATTN_XCD=0" "TCX_LB_RING=2" "TCX_SKIP_CM=3"; do
  echo "== $v" >> gpurun_out/${T}_c5.log
  env $v timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1 >> gpurun_out/${T}_c5.log 2>&1 || exit 1
done
bash tools/gpu/r05t.sh ${T}_t || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python3 bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 0 --lanes 1 --n-steps 12 > gpurun_out/${T}_prof.log 2>&1 || exit 1
python3 tools/rocpd_layers.py $(find gpurun_out/${T}_prof -name "*.db" | head -1) gpurun_out/${T}_cfg5_layers.txt
rm -rf gpurun_out/${T}_prof
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --fp32-passes 0 > gpurun_out/${T}_bench.log 2>&1 || exit 1
step timeout -k 10 900 $P tests/test_gpu_dp_scripts.py > gpurun_out/${T}_t4.log 2>&1
