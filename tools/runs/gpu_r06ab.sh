# round 6: scheduler options on top of the AMDGPU register-pressure trackers (hooks builds):
# metric bias 0 / 50, no unclustered high-RP reschedule, no clustered low-occupancy
# reschedule; kbench C3 / C4 2^20, hashes, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06ab_kb_sched2.log
: > $L
S=$V/mainhooks.so:$V/trackers.so:$V/t_bias0.so:$V/t_bias50.so:$V/t_norp.so:$V/t_nocl.so
for cfg in C3_ntru512 C4_qary1024; do
  echo "== $cfg" >> $L
  LGS_LIBS=$S:$S timeout -k 10 400 python tools/kbench.py --config $cfg --n 1048576 --reps 3 --hash 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
cat $L
