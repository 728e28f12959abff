# the q-panel skip's code in its own instantiation (default: launched only when a panel
# is skippable) vs the previous single instantiation (base) and a build without it (noqs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
L=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so:$V/base.so:$V/noqs.so
for cfg in C1_Z64 C2_qary128 C4_qary1024 C3_ntru512; do
  echo "== $cfg" && for r in 1 2; do LGS_LIBS=$L timeout -k 10 300 python tools/kbench.py --config $cfg --n 262144 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-230 || exit 1; done
done
