# round 6 final build (3ab9df7a, CU split): per-config Klein throughput (tools/bench_configs.py) and the bench's
# other workloads (C4 -- the 8-GPU config --, C5, C2) through bench.py --config
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r06bi
python3 -c "import hashlib; print('build', hashlib.sha256(open('lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so','rb').read()).hexdigest()[:16])" | tee gpurun_out/${TAG}_bench_configs.log
echo "== bench_configs" && timeout -k 10 600 python -u tools/bench_configs.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/${TAG}_bench_configs.log | cut -c1-300 || exit 1
for c in C4_qary1024 C5_ntru2048 C2_qary128; do
  echo "== $c"
  timeout -k 10 400 python bench.py --config $c --no-cpu --wl-steps 1 --steps 4 --warmup 1 > gpurun_out/${TAG}_$c.log 2>&1 || { tail -20 gpurun_out/${TAG}_$c.log; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/${TAG}_$c.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernel_ms']; print('$c', j['value'], j['ms_per_step'], j['config']['imhk_steps_per_step'], {x: k[x] for x in ('klein','bz','accept','moments')}, j['parity_check'], j['wang_ling']['value'], j['wang_ling']['flags_equal_oracle'][:60])"
done | tee gpurun_out/${TAG}_configs.log
# the 8-GPU command rehearsed with 2 ranks on one GPU (gloo), C4
echo "== 2 ranks C4"
LGS_ONE_DEVICE=1 LGS_DIST_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --config C4_qary1024 --steps 2 --warmup 1 > gpurun_out/r06bi_bench_2ranks_1gpu_C4.log 2>&1; rc=$?
tail -n 1 gpurun_out/r06bi_bench_2ranks_1gpu_C4.log | cut -c1-1500
exit $rc
