# Round 4 closing check at HEAD: smoke(), the bench line (with the re-measured traffic constant).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r04_close
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1
