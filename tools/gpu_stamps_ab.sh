set -o pipefail
mkdir -p gpurun_out
for seed in 1000 2000 3000 4000; do
  timeout -k 10 120 python tools/phase_stamps.py 1024 10 trot10 $seed > gpurun_out/sab_A_$seed.txt 2>&1 || exit 1
  MPCQP_STAMPS_LIB=pympc-quadruped_amd/mpcqp/libmpcqp_stamps_nopair.so timeout -k 10 120 python tools/phase_stamps.py 1024 10 trot10 $seed > gpurun_out/sab_B_$seed.txt 2>&1 || exit 1
done
grep -h "B=\|total\|slow\|cycles / iteration" gpurun_out/sab_*
