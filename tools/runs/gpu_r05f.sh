# round 5: Klein A/B of stacked near-field trims: tail2 (range checks from the
# sub-panel's extremes, row-base Z stores), t2dd (+ host dispatch code), t2d (+
# branchless quantile test), t2dh (+ per-coordinate history stores), t2df (+ capped
# kind first); C4 / C5 for the candidates
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
M=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
echo "== kbench C3" && for r in 1 2; do LGS_LIBS=$M:$V/tail2.so:$V/t2dd.so:$V/t2d.so:$V/t2dh.so:$V/t2df.so:$V/pnext.so:$V/t2dn.so timeout -k 10 400 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1; done | tee gpurun_out/r05f_kb.log
echo "== kbench C4 C5 C2" && for c in "C4_qary1024 262144" "C5_ntru2048 65536" "C2_qary128 262144"; do set -- $c; LGS_LIBS=$M:$V/t2dd.so:$V/t2d.so timeout -k 10 300 python tools/kbench.py --config $1 --n $2 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1; done | tee gpurun_out/r05f_kb45.log
echo "== wl C3" && LGS_LIBS=$M:$V/t2dd.so:$V/t2d.so timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 3 --hash --wl 2>&1 | grep -v amdgpu.ids | cut -c1-260 | tee gpurun_out/r05f_kbwl.log
