# round 5: moment partials reduced over DPP rows (row_ror) instead of LDS permutes, the
# column reduction on 4x more workgroups -- GPU suite, bench (isolated launches and default)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05w}
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "^E \|Error" gpurun_out/${TAG}_pytest_gpu.log | head -80; exit $rc; }
for r in 1 2; do for m in "LGS_NO_PIPE=1" "LGS_NO_PIPE=0"; do
  echo "== $m"
  env $m timeout -k 10 300 python bench.py --no-cpu --wl-steps 0 --steps 10 > gpurun_out/${TAG}_b.log 2>&1 || { tail -20 gpurun_out/${TAG}_b.log; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/${TAG}_b.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernel_ms']; print('$m', j['value'], j['ms_per_step'], {x: k[x] for x in ('klein','bz','accept','moments')}, j['parity_check'], j['covariance']['sum_zzT_sha256'])"
done; done | tee gpurun_out/${TAG}_bench_ab.log
