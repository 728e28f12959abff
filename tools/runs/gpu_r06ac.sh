# round 6 (rerun with mainhooks rebuilt from the current sources): the bench (isolated launches and pipelined) with the scheduler's register-pressure
# trackers + metric bias 50 (t_bias50) against the product's sources (mainhooks), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06ac_bench_sched.log
: > $L
for pipe in 1 0; do for rep in 1 2; do for v in mainhooks t_bias50; do
  echo "== $v no_pipe=$pipe" >> $L
  LGS_NO_PIPE=$pipe LGS_LIB=$V/$v.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'parity': d.get('parity_check')[:40]}))" >> $L || exit 1
done; done; done
cat $L
