set -o pipefail
cd $GRAFT_REPO_ROOT
V=lattice-gaussian-mcmc_amd/build/var

LGS_LIBS=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so:$V/diag_NO_SAMPLEZ.so:$V/diag_NO_FAR.so:$V/diag_NONE.so timeout -k 10 300 python tools/kbench.py --reps 3 2>&1 | grep -v amdgpu.ids
