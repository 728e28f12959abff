# Klein: the coordinate's uniform drawn under the record's LDS reads (default) vs after
# the kind tests (nopreu); output hashes must agree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
L=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so:$V/nopreu.so
for cfg in C3_ntru512 C2_qary128 C4_qary1024; do
  echo "== $cfg" && for r in 1 2; do LGS_LIBS=$L timeout -k 10 300 python tools/kbench.py --config $cfg --n 262144 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1; done
done
echo "== wl" && LGS_LIBS=$L timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 3 --hash --wl 2>&1 | grep -v amdgpu.ids | cut -c1-260
echo "== latency ubench" && timeout -k 10 120 ./tools/ubench/latency
