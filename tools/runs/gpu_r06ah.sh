# round 6: codegen options on top of the scheduler flags (hooks builds; mainhooks = the
# product's flags): wave priority, partial-reg-use rewrite, kernarg preload, speed-mode
# spill splitting, DCE in RA, memory clauses of 32, no loop alignment, relaxed occupancy;
# the pipelined bench, alternating, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06ah_bench_opts.log
: > $L
for rep in 1 2; do for v in mainhooks o_prio o_rewr o_kpre o_splitspd mainhooks o_dce o_clause o_noalign o_relax; do
  echo "== $v" >> $L
  LGS_LIB=$V/$v.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'parity': d.get('parity_check')[:40]}))" >> $L || exit 1
done; done
cat $L
