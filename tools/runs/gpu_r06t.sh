# round 6: same-box rocprof A/B of the B z change (mainhooks = the product's sources, bzold =
# 8-byte stores with the moments ahead of the MFMAs), isolated launches, kernel stats per run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp LGS_NO_PIPE=1
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06t_bz_rocprof_ab.log
: > $L
for rep in 1 2 3; do for v in bzold mainhooks; do
  O=gpurun_out/r06t_$v$rep
  LGS_LIB=$V/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 > $O.log 2>&1 || exit 1
  f=$(find $O -name run_kernel_stats.csv | head -1)
  echo "$v rep$rep $(grep -h 'bz_i8_kernel<short>' $f | awk -F'"' '{print $3}' | cut -d, -f2-5) klein $(grep -h 'klein_mfma_kernel<short, 32, false, true, false>' $f | awk -F'"' '{print $3}' | cut -d, -f2-5)" >> $L
done; done
cat $L
