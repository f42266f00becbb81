# Round 5 start: the headline-pinning / ABI tests, then the whole GPU suite and the bench line.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_a}
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_headline.py tests/test_gpu_models.py -k "headline or trained_sde300 or four_lanes or corun or error_path or workspace" > gpurun_out/${T}_new_tests.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1
