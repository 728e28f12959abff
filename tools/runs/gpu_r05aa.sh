# round 5: IMHK steps per bench step (one lgs_imhk call): 64 (one 2^20-proposal block),
# 128 in two 2^20 blocks, 128 in one 2^21 block (LGS_MAX_PROPOSALS) -- bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05aa}
for r in 1 2; do for m in "64 0" "128 0" "128 2097152"; do set -- $m
  echo "== imhk-steps $1 max-proposals $2"
  if [ "$2" != "0" ]; then export LGS_MAX_PROPOSALS=$2; else unset LGS_MAX_PROPOSALS; fi
  timeout -k 10 300 python bench.py --no-cpu --wl-steps 0 --steps 10 --imhk-steps $1 > gpurun_out/${TAG}_b.log 2>&1 || { tail -20 gpurun_out/${TAG}_b.log; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/${TAG}_b.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernel_ms']; print('$1 $2', j['value'], j['ms_per_step'], {x: k[x] for x in ('klein','bz','accept','moments')}, j['parity_check'])"
done; done | tee gpurun_out/${TAG}_bench_ab.log
