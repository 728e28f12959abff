# round 6: Klein-kernel A/B (bitop3 Philox, batch pins) and cost probes (far field, history, coupling reload)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
V=lattice-gaussian-mcmc_amd/build/var
LGS_LIBS=$L:$V/nobitop3.so:$V/pinbatch.so:$V/nofar.so:$V/farnomfma.so:$V/histfixed.so:$V/couplenoload.so:$L:$V/nobitop3.so timeout -k 10 400 python tools/kbench.py --config C3_ntru512 --n 1048576 --reps 3 --hash 2>&1 | grep -v amdgpu.ids || exit 1
LGS_LIBS=$L:$V/nobitop3.so:$L:$V/nobitop3.so timeout -k 10 300 python tools/kbench.py --config C4_qary1024 --n 1048576 --reps 2 --hash 2>&1 | grep -v amdgpu.ids
