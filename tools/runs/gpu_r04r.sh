# pre-drawn uniform debug: which part changes the outputs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
L=$V/nopreu.so:$V/dbg1.so:$V/dbg2.so
LGS_LIBS=$L timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 65536 --reps 1 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260
