# Config 3's workload on one GPU: the reference README recipe (README.md:95,104) through the
# mirror scripts — 50k rot-only dataset, 40 epochs, bs 128, lr 1e-4, beta 0.1-30, p_uncond 0.1,
# EMA 0.999 — then metrics.jsonl, the sample grid and the EMA weights back under gpurun_out/.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=$1
R=/tmp/recipe_$T
mkdir -p $R
timeout -k 10 300 python -u vae-diffusion-toy-crystals_amd/scripts/build_dataset.py --out $R/data.pt \
  --n-samples 50000 --img-size 64 --n-types 4 --rot-only > gpurun_out/${T}_build.log 2>&1 && \
timeout -k 10 1000 python -u vae-diffusion-toy-crystals_amd/scripts/train_sde_score_model.py --data-path $R/data.pt \
  --out-dir $R/run --epochs 40 --batch-size 128 --lr 1e-4 --beta-min 0.1 --beta-max 30 --p-uncond 0.1 \
  --ema-decay 0.999 > gpurun_out/${T}_train.log 2>&1 && \
cp $R/run/metrics.jsonl gpurun_out/${T}_metrics.jsonl && \
cp $R/run/results/*.png gpurun_out/ && \
python tools/export_ckpt.py $R/run/checkpoints/sde_score_model_last.pt gpurun_out/${T}_ema.npz ema
