# round 5: B z moments x pipelined blocks x Klein-stream priority (bench A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r05o
for r in 1 2; do for m in "LGS_NO_BZ_MOMENTS=1" "LGS_PIPE_PRIO=1" "LGS_PIPE_PRIO=2" "LGS_NO_PIPE=1"; do
  echo "== $m"
  env $m timeout -k 10 300 python bench.py --no-cpu --wl-steps 0 --steps 10 > gpurun_out/${TAG}_b.log 2>&1 || { tail -20 gpurun_out/${TAG}_b.log; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/${TAG}_b.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernel_ms']; print('$m', j['value'], j['ms_per_step'], {x: k[x] for x in ('klein','bz','accept','moments')}, j['parity_check'])"
done; done | tee gpurun_out/${TAG}_bench_ab.log
