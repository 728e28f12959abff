# round 5: Klein A/B (main = three-address near-field FMAs; capfma = + kind dispatch
# skipped in all-capped sub-panels), near-field step phase cycles (diagnostic
# builds), the round-4 dbg1 hazard rebuilt from the round-4 source (9b21303: its
# Philox v_mad_u64_u32 form and scalar-loaded erfinv coefficients)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
M=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
echo "== kbench C3" && for r in 1 2; do LGS_LIBS=$M:$V/capfma.so timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1; done | tee gpurun_out/r05c_kb.log
echo "== cycles" && LGS_LIBS=$V/diagcyc.so:$V/diagstep.so timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 2 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05c_cycles.log || exit 1
P=lattice-gaussian-mcmc_amd/build/r04pkg
echo "== r04 hazard" && LGS_LIBS=$P/lattice-gaussian-mcmc_amd/build/var/r4base.so:$P/lattice-gaussian-mcmc_amd/build/var/r4dbg1.so:$P/lattice-gaussian-mcmc_amd/build/var/r4dbg1b.so timeout -k 10 400 python $P/tools/kbench.py --config C3_ntru512 --n 65536 --reps 1 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-300 | tee gpurun_out/r05c_r04_hazard.log || exit 1
echo "== kbench C4 C5" && for c in "C4_qary1024 262144" "C5_ntru2048 65536"; do set -- $c; LGS_LIBS=$M:$V/capfma.so timeout -k 10 300 python tools/kbench.py --config $1 --n $2 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1; done | tee gpurun_out/r05c_kb45.log
