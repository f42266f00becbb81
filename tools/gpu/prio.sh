# s_setprio around the MFMA clusters of k_conv3p: one-lane bench A/B on one box (alternating)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
for i in 1 2; do
TCX_HALO_PRIO=1 timeout -k 10 200 python -u bench.py --steps 2 --lanes 1 --no-cpu-baseline > gpurun_out/$1_prio_$i.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 2 --lanes 1 --no-cpu-baseline > gpurun_out/$1_def_$i.log 2>&1 || exit 1
done
TCX_HALO_PRIO=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_h2.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$1_prio_tests.log 2>&1
