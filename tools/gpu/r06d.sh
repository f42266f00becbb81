# Round 6: training-step measurements — score / CondVAE / prior / DDIM-50 (three prior runs in one process
# each, for the box-to-box spread question), then a kernel trace of the score step for its breakdown.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_d}
STEPS=10 WARM=3 timeout -k 10 300 python -u tools/train_bench.py score vae prior ddim > gpurun_out/${T}_train.log 2>&1 || exit 1
for i in 1 2 3; do STEPS=30 WARM=5 timeout -k 10 120 python -u tools/train_bench.py prior >> gpurun_out/${T}_prior_runs.log 2>&1 || exit 1; done
STEPS=3 WARM=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_score -o run -- python3 tools/train_bench.py score > gpurun_out/${T}_score_prof.log 2>&1 || exit 1
STEPS=10 WARM=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prior -o run -- python3 tools/train_bench.py prior > gpurun_out/${T}_prior_prof.log 2>&1 || exit 1
for d in score prior; do
  cp "$(find gpurun_out/${T}_$d -name "*kernel_stats.csv" | head -1)" gpurun_out/${T}_${d}_kernel_stats.csv || exit 1
  rm -rf gpurun_out/${T}_$d
done
