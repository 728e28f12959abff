# round 5: Klein record layout L2 (decision fields first, near-field coefficients last and
# unpinned: the step waits for 16 of the record's 23 reads) -- kbench A/B with hashes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
M=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
TAG=r05af
echo "== kbench C3" && for r in 1 2; do LGS_LIBS=$M:$V/recl2.so timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1; done | tee gpurun_out/${TAG}_kb.log
echo "== kbench C4 C5 C2" && for c in "C4_qary1024 262144" "C5_ntru2048 65536" "C2_qary128 262144"; do set -- $c; LGS_LIBS=$M:$V/recl2.so timeout -k 10 300 python tools/kbench.py --config $1 --n $2 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1; done | tee gpurun_out/${TAG}_kb245.log
