# bench.py A/B over library variants (LGS_LIB), alternating: VARIANTS="main v ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in ${VARIANTS:-main}; do
  if [ $v = main ]; then f=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so; else f=lattice-gaussian-mcmc_amd/build/var/$v.so; fi
  LGS_LIB=$f timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_ab_$v.log 2>&1 || { tail -5 gpurun_out/bench_ab_$v.log; exit 1; }
  tail -1 gpurun_out/bench_ab_$v.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$v', json.dumps({k: j[k] for k in ('value','ms_per_step','kernel_ms','parity_check')}))"
done
