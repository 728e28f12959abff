# moments pass: two vectors per lane and pass (momu2) vs one (momu1, the previous loop);
# bench parity line and covariance checksum must agree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
for r in 1 2; do for lib in $V/momu2.so $V/momu1.so; do
echo "== $lib" && LGS_LIB=$lib timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r04u_b.log 2>&1 || { tail -5 gpurun_out/r04u_b.log; exit 1; }
tail -1 gpurun_out/r04u_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['parity_check'], d['covariance']['sum_zzT_sha256'], d['autocorrelation']['z_last'][1])"
done; done
