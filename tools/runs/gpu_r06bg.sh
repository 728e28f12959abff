# round 6: B z variants under the CU split (B z on 32 CUs beside the Klein launch is the
# step's critical path, r06bf_timeline.log): 64-coordinate tiles, 4 workgroups per CU,
# 2 tiles per workgroup, against the hooks build of the product; pipelined bench, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06bg_bench_bz_variants.log
: > $L
for rep in 1 2; do for v in main bn64 occ4 txper2; do
  lib=$V/$v.so; [ $v = main ] && lib=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip_hooks.so
  echo "== $v" >> $L
  LGS_LIB=$lib timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'cus': k.get('klein_stream_cus'), 'parity': d.get('parity_check')[:40]}))" >> $L || exit 1
done; done
cat $L
