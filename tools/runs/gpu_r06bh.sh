# round 6: B z on its own stream masked to the 32 CUs the Klein stream leaves out
# (hooks LGS_PIPE_BZ_MASK=1), with the product's B z tiles (mainh), 64-coordinate tiles
# (bn64) and four workgroups per CU (occ4); baseline mainh without the mask; two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06bh_bench_bzmask.log
: > $L
for rep in 1 2; do for cfg in "mainh 0" "mainh 1" "bn64 1" "occ4 1"; do
  set -- $cfg
  echo "== $1 bz_mask=$2" >> $L
  LGS_PIPE_BZ_MASK=$2 LGS_LIB=$V/$1.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'cus': k.get('klein_stream_cus'), 'parity': d.get('parity_check')[:40]}))" >> $L || exit 1
done; done
cat $L
