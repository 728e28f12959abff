# round 6: the combination (record reads unpinned + Philox keys hoisted + decision-first
# record, c_all) against the product's sources: kbench hashes and speed C1 .. C5 and
# Wang-Ling C3, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06av_call_kbench.log
: > $L
S=$V/mainhooks.so:$V/c_all.so
for c in "C1_Z64 1048576" "C2_qary128 1048576" "C3_ntru512 1048576" "C4_qary1024 1048576" "C5_ntru2048 131072"; do set -- $c
  echo "== kbench $1" >> $L
  LGS_LIBS=$S:$S timeout -k 10 300 python tools/kbench.py --config $1 --n $2 --reps 3 --hash 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
echo "== kbench C3 wl" >> $L
LGS_LIBS=$S:$S timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 3 --hash --wl 2>&1 | grep -v amdgpu.ids >> $L || exit 1
cat $L
