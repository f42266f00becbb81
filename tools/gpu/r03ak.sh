# prior DDIM-50: host-issued native call vs the same call graph-captured and replayed
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=r03_ak
timeout -k 10 300 python -u tools/ddim_graph_probe.py > gpurun_out/${T}_ddim_graph.log 2>&1
