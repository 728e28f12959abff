# Wang-Ling Klein: ln of the capped window sum by ln_fast (SGPR constants) vs ocml log;
# z hashes must agree (the log weights differ in the last bits, within the bounds)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
echo "== wl tests (lnfast)" && LGS_LIB=$V/lnfast.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wl_accept.py tests/test_gpu_configs.py tests/test_gpu_certificate.py 2>&1 | tail -1 || exit 1
L=$V/final.so:$V/lnfast.so
for cfg in C3_ntru512 C4_qary1024; do
  echo "== wl $cfg" && for r in 1 2; do LGS_LIBS=$L timeout -k 10 300 python tools/kbench.py --config $cfg --n 262144 --reps 5 --hash --wl 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1; done
done
