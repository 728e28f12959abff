# round 6: same-box bench A/B of the final build's q-skip (mainhooks = the same sources as the
# product, hooks build) against the staged q-panels (qstaged), isolated and pipelined; then the
# 2-rank rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
: > gpurun_out/r06p_bench_ab.log
for rep in 1 2; do for v in mainhooks qstaged; do
  echo "== $v" >> gpurun_out/r06p_bench_ab.log
  LGS_LIB=$V/$v.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein_ms': d['kernel_ms']['klein'], 'build': d['roofline']['build_id'], 'parity': d.get('parity')}))" >> gpurun_out/r06p_bench_ab.log || exit 1
done; done
cat gpurun_out/r06p_bench_ab.log
bash tools/runs/gpu_r06o.sh
