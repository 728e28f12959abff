# round 5: VALU issue rates (tools/ubench/valu_rates.hip); near-field decision cost
# probes (diagnostic, NOT bit-exact builds): Philox -> 4-instruction hash (cheaprng),
# capped decision = its quantile guess (capguess), with and without step-phase cycles
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
M=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
echo "== valu rates" && timeout -k 10 120 ./tools/ubench/valu_rates 2>&1 | tee gpurun_out/r05d_valu_rates.log || exit 1
echo "== probes" && LGS_LIBS=$M:$V/cheaprng.so:$V/capguess.so:$V/diagstep.so:$V/stepcheap.so:$V/stepguess.so timeout -k 10 400 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 2>&1 | grep -v amdgpu.ids | cut -c1-900 | tee gpurun_out/r05d_probes.log || exit 1
