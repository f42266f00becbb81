# HBM traffic per conv launch for config 5 (256^2 bf16, 2-byte tensors): separate rocprofv3 --pmc FETCH_SIZE /
# WRITE_SIZE passes over the one-lane pass of bench.py's config-5 line (Bt = 128 per launch), two sampler steps.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r05_t}
A="--img-size 256 --batch 64 --precision bf16 --n-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --lanes 1"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch -o p -- python3 bench.py $A > gpurun_out/${T}_fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write -o p -- python3 bench.py $A > gpurun_out/${T}_write.log 2>&1 && \
python3 tools/pmc_traffic.py gpurun_out/${T}_fetch gpurun_out/${T}_write > gpurun_out/${T}_pmc_traffic.txt 2>&1 && \
rm -rf gpurun_out/${T}_fetch gpurun_out/${T}_write
