# k_conv3l per-workgroup phase stamps (tools/conv3l_stamps.py) at the up1_1 shape
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
TCX_CONV3L_DBG=1 timeout -k 10 120 python3 tools/conv3l_stamps.py > gpurun_out/${T}_dbg1.log 2>&1 && \
TCX_CONV3L_DBG=2 timeout -k 10 120 python3 tools/conv3l_stamps.py > gpurun_out/${T}_dbg2.log 2>&1 && \
TCX_CONV3L_DBG=1 CIN=192 timeout -k 10 120 python3 tools/conv3l_stamps.py > gpurun_out/${T}_dbg1_c192.log 2>&1
