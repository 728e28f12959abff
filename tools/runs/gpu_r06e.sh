# round 6: far-field cost probes (C3, 2^20 proposals): no MFMA, no slab, fixed history; coupling reload
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
V=lattice-gaussian-mcmc_amd/build/var
LGS_LIBS=$L:$V/farnomfma.so:$V/farnoslab.so:$V/histfixed.so:$V/couplenoload.so:$L timeout -k 10 400 python tools/kbench.py --config C3_ntru512 --n 1048576 --reps 3 2>&1 | grep -v amdgpu.ids
