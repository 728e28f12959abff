# Far-field digit count sweep: kbench (Klein + B z) of the default library and the
# LGS_OZ_DIGITS variants, then the bench (certificate redo counts) with each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
VARIANTS="main ${OZ_VARIANTS:-oz5 oz4}" bash tools/gpu_kb.sh || exit 1
for v in ${OZ_VARIANTS:-oz5 oz4}; do
  echo "== bench $v"
  LGS_LIB=$V/$v.so timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_$v.log 2>&1 || { tail -5 gpurun_out/bench_$v.log; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/bench_$v.log') if x.startswith('{')][-1]; j=json.loads(l); print(json.dumps({k: j[k] for k in ('value','parity_check','certificate_redos','kernel_ms')}))"
done
