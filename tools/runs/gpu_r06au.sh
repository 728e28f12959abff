# round 6: the small gains combined: record reads unpinned (c_np), + Philox keys hoisted
# (c_np_ph), + decision-first record (c_np_l2), all three (c_all); hooks builds, mainhooks = the product;
# pipelined bench, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06au_bench_variants.log
: > $L
for rep in 1 2 3; do for v in mainhooks c_np c_np_ph c_np_l2 c_all; do
  echo "== $v" >> $L
  LGS_LIB=$V/$v.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'parity': d.get('parity_check')[:40]}))" >> $L || exit 1
done; done
cat $L
