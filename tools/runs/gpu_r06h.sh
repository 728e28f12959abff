# round 6: far field with the R-digit fragments loaded straight from global memory (no LDS slab,
# no block barriers), ring of 4 / 6 / 8 fragments, vs the LDS-staged slab (main); C3 and C4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
V=lattice-gaussian-mcmc_amd/build/var
LGS_LIBS=$L:$V/direct4.so:$V/direct6.so:$V/direct8.so:$L timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 1048576 --reps 3 --hash 2>&1 | grep -v amdgpu.ids || exit 1
LGS_LIBS=$L:$V/direct6.so:$V/direct8.so timeout -k 10 300 python tools/kbench.py --config C4_qary1024 --n 1048576 --reps 2 --hash 2>&1 | grep -v amdgpu.ids
