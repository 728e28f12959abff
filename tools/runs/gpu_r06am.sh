# round 6: more kept-out variants re-screened under the scheduler flags and the capped
# sub-panel default (hooks builds; mainhooks = the product's sources): Philox variants
# (next / hoist / two blocks), capped dispatch first, batch-pinned record, B z two tiles per
# workgroup, decision-first record, near field unrolled by two; pipelined bench, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06am_bench_variants.log
: > $L
for rep in 1 2; do for v in mainhooks w_philnext w_philhoist w_philox2 w_dispfirst mainhooks w_pinbatch w_bztx2 w_recl2 w_unroll2; do
  echo "== $v" >> $L
  LGS_LIB=$V/$v.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'parity': d.get('parity_check')[:40]}))" >> $L || exit 1
done; done
cat $L
