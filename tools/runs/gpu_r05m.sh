# round 5: the kept states' moments from B z's digit tiles (bz_i8 MP partials + a column
# reduction, final states from the int16 history) -- GPU suite, bench A/B against the
# separate moments pass (LGS_NO_BZ_MOMENTS=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05m}
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "^E \|Error" gpurun_out/${TAG}_pytest_gpu.log | head -80; exit $rc; }
for r in 1 2; do for m in "LGS_NO_BZ_MOMENTS=1" "LGS_NO_BZ_MOMENTS=0" "LGS_NO_PIPE=1"; do
  echo "== $m"
  env $m timeout -k 10 300 python bench.py --no-cpu --wl-steps 0 --steps 10 > gpurun_out/${TAG}_b.log 2>&1 || { tail -20 gpurun_out/${TAG}_b.log; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/${TAG}_b.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernel_ms']; print('$m', j['value'], j['ms_per_step'], {x: k[x] for x in ('klein','bz','accept','moments')}, j['parity_check'], j['covariance']['sum_zzT_sha256'], j['autocorrelation']['z_last'][1])"
done; done | tee gpurun_out/${TAG}_bench_ab.log
