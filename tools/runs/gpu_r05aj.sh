# round 5: the bench's other workloads at the new defaults (256 IMHK steps per call,
# 2^22-proposal cap): C4 (the 8-GPU config, two blocks per call), C5 (d = 4096), C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r05aj
for c in C4_qary1024 C5_ntru2048 C2_qary128; do
  echo "== $c"
  timeout -k 10 400 python bench.py --config $c --no-cpu --wl-steps 1 --steps 4 --warmup 1 > gpurun_out/${TAG}_$c.log 2>&1 || { tail -20 gpurun_out/${TAG}_$c.log; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/${TAG}_$c.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernel_ms']; print('$c', j['value'], j['ms_per_step'], j['config']['imhk_steps_per_step'], {x: k[x] for x in ('klein','bz','accept','moments')}, j['parity_check'], j['wang_ling']['value'], j['wang_ling']['flags_equal_oracle'][:60])"
done | tee gpurun_out/${TAG}_configs.log
