# round 6: LLVM scheduler options for the whole library (hooks builds): the AMDGPU register
# pressure trackers (trackers), the max-memory-clause strategy (memclause) against the
# product's sources (mainhooks); kbench C3 / C4 2^20, hashes, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06aa_kb_sched.log
: > $L
for cfg in C3_ntru512 C4_qary1024; do
  echo "== $cfg" >> $L
  LGS_LIBS=$V/mainhooks.so:$V/trackers.so:$V/memclause.so:$V/mainhooks.so:$V/trackers.so:$V/memclause.so timeout -k 10 300 python tools/kbench.py --config $cfg --n 1048576 --reps 3 --hash 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
cat $L
