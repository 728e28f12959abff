# round 6: the look-ahead Klein launch enqueued right behind the call's last Klein launch
# (hooks LGS_LOOKAHEAD_EARLY=1) under the CU split -- the Klein stream otherwise idles
# ~2 ms per step until the host reads flag words queued behind B z (r06bf_timeline.log)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
H=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip_hooks.so
L=gpurun_out/r06bj_bench_look_early.log
: > $L
for rep in 1 2; do for e in 0 1; do
  echo "== lookahead_early=$e" >> $L
  LGS_LOOKAHEAD_EARLY=$e LGS_LIB=$H timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'cus': k.get('klein_stream_cus'), 'parity': d.get('parity_check')[:40]}))" >> $L || exit 1
done; done
cat $L
