# round 5: Klein A/B -- tail3 (integer extremes, running history pointer, the
# uncovered-decision mask behind a ballot, scalar dispatch word) and, on top of it,
# the round-4 Philox form (v_mad_u64_u32, t3mad) and an Estrin erfinv (t3est)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
M=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
echo "== kbench C3" && for r in 1 2; do LGS_LIBS=$M:$V/tail3.so:$V/t3mad.so:$V/t3est.so timeout -k 10 400 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1; done | tee gpurun_out/r05h_kb.log
echo "== kbench C4 C5" && for c in "C4_qary1024 262144" "C5_ntru2048 65536"; do set -- $c; LGS_LIBS=$M:$V/tail3.so timeout -k 10 300 python tools/kbench.py --config $1 --n $2 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1; done | tee gpurun_out/r05h_kb45.log
