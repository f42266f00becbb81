# k_conv3p with 8 waves / 256-pixel tiles (TCX_HALO_PNW=8): parity, then one-lane bench A/B (alternating)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TCX_HALO_PNW=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$1_pnw8_tests.log 2>&1 || exit 1
for i in 1 2; do
TCX_HALO_PNW=8 timeout -k 10 200 python -u bench.py --steps 2 --lanes 1 --no-cpu-baseline > gpurun_out/$1_pnw8_$i.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 2 --lanes 1 --no-cpu-baseline > gpurun_out/$1_def_$i.log 2>&1 || exit 1
done
