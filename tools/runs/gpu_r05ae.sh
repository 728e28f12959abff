# round 5: 256 vs 512 IMHK steps per bench step (512: two 2^22-proposal blocks per call)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05ae}
for r in 1 2; do for m in 256 512; do
  echo "== imhk-steps $m"
  timeout -k 10 300 python bench.py --no-cpu --wl-steps 0 --steps 6 --warmup 2 --imhk-steps $m > gpurun_out/${TAG}_b.log 2>&1 || { tail -20 gpurun_out/${TAG}_b.log; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/${TAG}_b.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernel_ms']; print('$m', j['value'], j['ms_per_step'], {x: k[x] for x in ('klein','bz','accept','moments')}, j['parity_check'])"
done; done | tee gpurun_out/${TAG}_bench_ab.log
