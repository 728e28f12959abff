# round 6: q-skipped panels without record staging (main) vs staged (qstaged); coarse panels staging
# only their 4 digits (main) vs the full slab (fullslab); C3 / C4 / C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
V=lattice-gaussian-mcmc_amd/build/var
LGS_LIBS=$L:$V/qstaged.so:$V/fullslab.so:$L:$V/qstaged.so:$V/fullslab.so timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 1048576 --reps 3 --hash 2>&1 | grep -v amdgpu.ids || exit 1
LGS_LIBS=$L:$V/qstaged.so:$V/fullslab.so:$L:$V/fullslab.so timeout -k 10 300 python tools/kbench.py --config C4_qary1024 --n 1048576 --reps 3 --hash 2>&1 | grep -v amdgpu.ids || exit 1
LGS_LIBS=$L:$V/fullslab.so timeout -k 10 300 python tools/kbench.py --config C5_ntru2048 --n 131072 --reps 2 --hash 2>&1 | grep -v amdgpu.ids
