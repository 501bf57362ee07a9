cd $GRAFT_REPO_ROOT
for N in 24 32; do for c in flight sparse trot standing; do
  timeout -k 5 40 python tools/diag_long_horizon.py $N $c > gpurun_out/diag_${N}_$c.txt 2>&1; echo "rc $? ($N $c)"; grep -v amdgpu.ids gpurun_out/diag_${N}_$c.txt | tail -3
done; done
