# round 6: the kept-out Klein variants re-screened under the scheduler flags (hooks builds;
# mainhooks = the product's sources): record decision-first (recl2), pipelined far-field
# passes (ozpipe), erfinv immediates (capimm), F tiles aliased with the slab (xpalias),
# all-capped sub-panel copy (capsp), Philox at the step's top (philtop); the pipelined
# bench, alternating, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06ak_bench_variants.log
: > $L
for rep in 1 2; do for v in mainhooks v_recl2 v_ozpipe v_capimm mainhooks v_xpalias v_capsp v_philtop; do
  echo "== $v" >> $L
  LGS_LIB=$V/$v.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'parity': d.get('parity_check')[:40]}))" >> $L || exit 1
done; done
cat $L
