# Round-6 final verification, part A: determinism (alone + co-run), the whole GPU suite, smoke, the bench line
# (with the CPU baseline) and config 5's bench line.  A test FAILURE (rc 1) does not stop the script; a
# timeout, abort or crash (rc >= 124) does.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_fin}
step() { "$@"; rc=$?; echo "rc=$rc: $*" >> gpurun_out/${T}_steps.log; if [ $rc -ge 124 ]; then exit $rc; fi; return 0; }
step timeout -k 10 200 python -u tools/determinism_probe.py > gpurun_out/${T}_det.log 2>&1
step timeout -k 10 200 python -u tools/determinism_probe.py --corun > gpurun_out/${T}_corun.log 2>&1
step timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
step timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1
step timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.log 2>&1
step timeout -k 10 300 python -u bench.py --img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${T}_c5.log 2>&1
