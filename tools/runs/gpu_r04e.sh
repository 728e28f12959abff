# Klein-kernel A/B of library variants (kbench, C3 2^18, alternating twice)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
LIBS=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so:$V/noq.so:$V/nock.so:$V/noqck.so:$V/r03.so
echo "== kbench A/B" && for r in 1 2; do LGS_LIBS=$LIBS timeout -k 10 400 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 || exit 1; done > gpurun_out/r04e_ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r04e_ab.log | cut -c1-160; exit $rc
