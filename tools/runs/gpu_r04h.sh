# B z bound probes: write bandwidth, store-only / no-store bz builds at 2^18 and 2^20
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
echo "== wbw" && timeout -k 10 120 python tools/diag/wbw.py || exit 1
L=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so:$V/bzstoreonly.so:$V/bznostore.so
for n in 262144 1048576; do
  echo "== n=$n" && LGS_LIBS=$L timeout -k 10 400 python tools/kbench.py --config C3_ntru512 --n $n --reps 4 --bz 2>&1 | grep -v amdgpu.ids | cut -c1-250 || exit 1
done
