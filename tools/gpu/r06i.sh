# Round 6: what holds MFMA busy at ~50 % in the GroupNorm-prologue conv (up1_1, k_conv3m PRO 1 vs the h2-source
# PRO 0 form on the same layer) and in config 5's k_conv3lb<256> / attention: VALU issue cycles, transcendental
# and conversion counts, LDS activity — two counter groups per kernel, one pass each.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-r06_i}
GA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
GB="SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
export H2=1 REPS=5 LAYER=up1_1
for P in 1 0; do
  export PRO=$P
  timeout -s KILL 90 rocprofv3 --pmc $GA --output-format csv -d gpurun_out/${T}_pro${P}_A -o p -- python3 tools/convone.py > gpurun_out/${T}_pro${P}_A.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $GB --output-format csv -d gpurun_out/${T}_pro${P}_B -o p -- python3 tools/convone.py > gpurun_out/${T}_pro${P}_B.log 2>&1 || exit 1
  echo "== k_conv3m PRO=$P up1_1" >> gpurun_out/${T}_pmc.txt
  python3 tools/pmc_summary.py "k_conv3m" gpurun_out/${T}_pro${P}_A gpurun_out/${T}_pro${P}_B >> gpurun_out/${T}_pmc.txt || exit 1
done
unset H2 REPS LAYER PRO
A="--img-size 256 --batch 64 --precision bf16 --no-cpu-baseline --steps 1 --warmup 0 --lanes 1 --n-steps 2"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_conv3lb<256|k_attention" --pmc $GA --output-format csv -d gpurun_out/${T}_c5_A -o p -- python3 bench.py $A > gpurun_out/${T}_c5_A.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_conv3lb<256|k_attention" --pmc $GB --output-format csv -d gpurun_out/${T}_c5_B -o p -- python3 bench.py $A > gpurun_out/${T}_c5_B.log 2>&1 || exit 1
for k in "k_conv3lb<256" "k_attention"; do
  echo "== $k (config 5)" >> gpurun_out/${T}_pmc.txt
  python3 tools/pmc_summary.py "$k" gpurun_out/${T}_c5_A gpurun_out/${T}_c5_B >> gpurun_out/${T}_pmc.txt || exit 1
done
tar czf gpurun_out/${T}_raw.tgz gpurun_out/${T}_pro* gpurun_out/${T}_c5_* && rm -rf gpurun_out/${T}_pro1_* gpurun_out/${T}_pro0_* gpurun_out/${T}_c5_A gpurun_out/${T}_c5_B
