# Round 6 last check of the in-tree library: smoke, the training / prior / bf16 tests and the default bench line.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_fin5}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
tail -n 1 gpurun_out/${T}_smoke.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_prior.py tests/test_gpu_bf16.py > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -n 1 gpurun_out/${T}_tests.txt
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 1
grep '^{' gpurun_out/${T}_bench.log | head -1 | cut -c1-200
