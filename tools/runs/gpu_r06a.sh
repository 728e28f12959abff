# round 6: LDS-aliased far field at 2 and 3 waves per SIMD (kbench A/B with output hashes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
V=lattice-gaussian-mcmc_amd/build/var
for cfg in "C3_ntru512 1048576" "C4_qary1024 262144"; do set -- $cfg
  LGS_LIBS=$L:$V/alias2.so:$V/alias3.so:$V/alias3ng1.so:$L:$V/alias3.so timeout -k 10 300 python tools/kbench.py --config $1 --n $2 --reps 3 --hash 2>&1 | grep -v amdgpu.ids || exit 1
done
