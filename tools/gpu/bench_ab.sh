# A/B of an env knob on the headline bench (after the split-path + model parity tests)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1; KNOB=$2; shift 2
timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit 1
for v in "$@"; do
  env $KNOB=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_bench_${v}.log 2>&1 || exit 1
done
