# Klein re-tune after the q-panel skip (the H half now dominates): one far-field group
# per pass (ng1), capped coefficients not pre-loaded (noripre), near field unrolled by
# 2 (unroll2), Philox with mul_hi (mulhi) vs the current build (base); hashes must agree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
L=$V/base.so:$V/ng1.so:$V/noripre.so:$V/unroll2.so:$V/mulhi.so
for cfg in C3_ntru512 C4_qary1024; do
  echo "== $cfg" && for r in 1 2; do LGS_LIBS=$L timeout -k 10 400 python tools/kbench.py --config $cfg --n 262144 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-230 || exit 1; done
done
