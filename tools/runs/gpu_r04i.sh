# bench with B z diagnostic variants (no ||v||^2 partials / no selections) vs the default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
for lib in lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so $V/bznovnp.so $V/bznosel.so; do
  echo "== $lib" && LGS_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --steps 6 > gpurun_out/r04i_b.log 2>&1 || { tail -5 gpurun_out/r04i_b.log; exit 1; }
  tail -1 gpurun_out/r04i_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'])"
done
