# round 5: Klein A/B -- Philox blocks of a quad of slots computed together (ph2), drawn
# under the record's LDS reads (ph2top), erfinv coefficients as scalar immediates
# (capimm), all three (allx); hashes must equal main's
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
M=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
echo "== kbench C3" && for r in 1 2; do LGS_LIBS=$M:$V/ph2.so:$V/ph2top.so:$V/capimm.so:$V/allx.so:$V/capbl.so:$V/disp.so timeout -k 10 400 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1; done | tee gpurun_out/r05e_kb.log
