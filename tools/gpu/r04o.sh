# Round 4: after the AGPR-form fix: co-run + 4-lane determinism, the whole GPU suite, bench, kernel trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r04_o}
timeout -k 10 200 python -u tools/determinism_probe.py > gpurun_out/${T}_det.log 2>&1 && \
timeout -k 10 200 python -u tools/determinism_probe.py --corun > gpurun_out/${T}_corun.log 2>&1 && \
grep -q "^deterministic" gpurun_out/${T}_det.log && grep -q "^deterministic" gpurun_out/${T}_corun.log && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes 1 --fp32-passes 0 > gpurun_out/${T}_prof.log 2>&1
