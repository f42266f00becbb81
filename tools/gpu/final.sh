# Round-5 final verification: determinism (alone + co-run), the whole GPU suite, smoke, the bench line
# (with the CPU baseline), config 5's bench line, kernel-trace stats of the one-lane pass, HBM traffic PMC
# passes at the roofline's configuration (one lane: Bt = 256 per launch), training steps and the DDIM
# kernel trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_fin}
timeout -k 10 200 python -u tools/determinism_probe.py > gpurun_out/${T}_det.log 2>&1 && \
timeout -k 10 200 python -u tools/determinism_probe.py --corun > gpurun_out/${T}_corun.log 2>&1 && \
grep -q "^deterministic" gpurun_out/${T}_det.log && grep -q "^deterministic" gpurun_out/${T}_corun.log && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${T}_c5.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch -o p -- python3 bench.py --n-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --fp32-passes 0 --lanes 1 > gpurun_out/${T}_fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write -o p -- python3 bench.py --n-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --fp32-passes 0 --lanes 1 > gpurun_out/${T}_write.log 2>&1 && \
python3 tools/pmc_traffic.py gpurun_out/${T}_fetch gpurun_out/${T}_write > gpurun_out/${T}_pmc_traffic.txt 2>&1 && \
STEPS=10 WARM=3 timeout -k 10 300 python -u tools/train_bench.py score vae prior ddim > gpurun_out/${T}_train.log 2>&1 && \
STEPS=3 WARM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_ddim -o run -- python3 tools/train_bench.py ddim > gpurun_out/${T}_ddim.log 2>&1
