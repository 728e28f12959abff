# round 6: next panel's records prefetched into registers (recpf) vs loaded at the staging (recnopf); C3 ref / WL, C4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
LGS_LIBS=$V/recpf.so:$V/recnopf.so:$V/recpf.so:$V/recnopf.so timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 1048576 --reps 3 --hash 2>&1 | grep -v amdgpu.ids || exit 1
LGS_LIBS=$V/recpf.so:$V/recnopf.so timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 3 --hash --wl 2>&1 | grep -v amdgpu.ids || exit 1
LGS_LIBS=$V/recpf.so:$V/recnopf.so timeout -k 10 300 python tools/kbench.py --config C4_qary1024 --n 1048576 --reps 3 --hash 2>&1 | grep -v amdgpu.ids
