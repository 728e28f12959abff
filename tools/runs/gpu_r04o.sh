# Klein cost probes of the current build (diagnostic, not bit-exact): no far field,
# capped decision = the quantile guess, neither
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
L=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so:$V/nofar.so:$V/capguess.so:$V/skel.so
echo "== probes" && LGS_LIBS=$L timeout -k 10 500 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 2>&1 | grep -v amdgpu.ids | cut -c1-200
