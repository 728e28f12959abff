# Bench the main library against diagnostic variants (lattice-gaussian-mcmc_amd/build/var/*.so),
# two alternating rounds: bash tools/gpu_cmp_variants.sh var1 var2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
for rep in 1 2; do
for lib in main "$@"; do
  if [ $lib = main ]; then unset LGS_LIB; else export LGS_LIB=$V/$lib.so; fi
  timeout -k 10 120 python bench.py --no-cpu > gpurun_out/cmp_$lib.log 2>&1 || { echo "fail $lib"; tail -20 gpurun_out/cmp_$lib.log; exit 1; }
  python -c "import json,sys; l=[x for x in open('gpurun_out/cmp_$lib.log') if x.startswith('{')][-1]; j=json.loads(l); print('$lib', j['value'], j['kernel_ms'], j['parity_check'], j.get('certificate_redos'))"
done
done
