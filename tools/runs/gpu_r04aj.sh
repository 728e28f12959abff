# cost probe (diagnostic, not bit-exact): the near-field coupling without its z loads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
echo "== probe" && for r in 1 2; do LGS_LIBS=$V/final.so:$V/nocpl.so timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 2>&1 | grep -v amdgpu.ids | cut -c1-200 || exit 1; done
