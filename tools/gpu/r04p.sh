# Round 4 final verification, part 1: determinism (alone + co-run), the whole GPU suite.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r04_p}
timeout -k 10 200 python -u tools/determinism_probe.py > gpurun_out/${T}_det.log 2>&1 && \
timeout -k 10 200 python -u tools/determinism_probe.py --corun > gpurun_out/${T}_corun.log 2>&1 && \
grep -q "^deterministic" gpurun_out/${T}_det.log && grep -q "^deterministic" gpurun_out/${T}_corun.log && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
