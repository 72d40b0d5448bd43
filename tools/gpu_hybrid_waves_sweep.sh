set -o pipefail
for hw in 4 8 16; do
  POLAR_SC_HYBRID_WAVES=$hw timeout -k 10 200 python -u tools/wpg_sweep.py --mask frozen_n_65536_k_32768 --batches 4096 --wpg 4,8,16 --reps 5 >> gpurun_out/t4_sweep.log 2>&1 || exit 1
  POLAR_SC_HYBRID_WAVES=$hw timeout -k 10 200 python -u tools/wpg_sweep.py --mask frozen_n_262144_k_131072 --batches 512,64 --wpg 4,8,16 --reps 3 >> gpurun_out/t4_sweep.log 2>&1 || exit 1
  echo "hw $hw done"
done
