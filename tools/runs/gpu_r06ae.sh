# round 6: more scheduler settings against trackers + metric bias 50 (t_bias50): bias 100
# (t_b100), bias 50 without the unclustered high-RP reschedule (t_b50norp), bias 50 without
# the trackers (b50only); the bench pipelined and isolated, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06ae_bench_sched.log
: > $L
for pipe in 0 1; do for v in t_bias50 t_b100 t_b50norp b50only t_bias50 mainhooks; do
  echo "== $v no_pipe=$pipe" >> $L
  LGS_NO_PIPE=$pipe LGS_LIB=$V/$v.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'parity': d.get('parity_check')[:40]}))" >> $L || exit 1
done; done
cat $L
