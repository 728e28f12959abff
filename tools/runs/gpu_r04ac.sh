# Philox with mul_hi (mulhi), and with the capped coefficients not pre-loaded (mulhiri),
# vs the current build (base), three alternating runs per config; hashes must agree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
L=$V/base.so:$V/mulhi.so:$V/mulhiri.so
for cfg in C3_ntru512 C4_qary1024 C2_qary128 C5_ntru2048; do
  n=262144; [ $cfg = C5_ntru2048 ] && n=65536
  echo "== $cfg" && for r in 1 2 3; do LGS_LIBS=$L timeout -k 10 400 python tools/kbench.py --config $cfg --n $n --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-230 || exit 1; done
done
echo "== wl" && LGS_LIBS=$L timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 3 --hash --wl 2>&1 | grep -v amdgpu.ids | cut -c1-230
