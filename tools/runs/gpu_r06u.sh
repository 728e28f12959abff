# round 6: Klein records through scalar loads at each use (recsmem), only the 15 near-field coefficients so (rssmem), against the product's
# sources (mainhooks): kbench C3 / C4 2^20, hashes, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06u_kb_recsmem.log
: > $L
for cfg in C3_ntru512 C4_qary1024; do
  echo "== $cfg" >> $L
  LGS_LIBS=$V/mainhooks.so:$V/recsmem.so:$V/rssmem.so:$V/mainhooks.so:$V/recsmem.so:$V/rssmem.so timeout -k 10 300 python tools/kbench.py --config $cfg --n 1048576 --reps 3 --hash 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
cat $L
