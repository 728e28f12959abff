# round 6: far-field passes pipelined as one sequence (main) vs split passes (round 5), C3 / C4 / C5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
V=lattice-gaussian-mcmc_amd/build/var
LGS_LIBS=$L:$V/splitpass.so:$L:$V/splitpass.so timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 1048576 --reps 3 --hash 2>&1 | grep -v amdgpu.ids || exit 1
LGS_LIBS=$L:$V/splitpass.so:$L:$V/splitpass.so timeout -k 10 300 python tools/kbench.py --config C4_qary1024 --n 1048576 --reps 3 --hash 2>&1 | grep -v amdgpu.ids || exit 1
LGS_LIBS=$L:$V/splitpass.so timeout -k 10 300 python tools/kbench.py --config C5_ntru2048 --n 131072 --reps 2 --hash 2>&1 | grep -v amdgpu.ids
