# Klein: near-field coefficients 2..14 through scalar loads (rsscalar: next to their
# FMAs; rsscalar2: with the record's reads) vs the LDS batch (base); hashes must agree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
L=$V/base.so:$V/rsscalar.so:$V/rsscalar2.so
for cfg in C3_ntru512 C4_qary1024 C2_qary128; do
  echo "== $cfg" && for r in 1 2; do LGS_LIBS=$L timeout -k 10 300 python tools/kbench.py --config $cfg --n 262144 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-230 || exit 1; done
done
