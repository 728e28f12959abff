# round 6: kernel timeline of the pipelined bench with the CU split (rocprofv3 kernel
# trace, tools/trace_timeline.py): split on, off, and on with three buffer sets (hooks
# build, LGS_PIPE_SETS=3); then bench A/B of the three sets without the profiler
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
H=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip_hooks.so
for mode in split nosplit sets3; do
  case $mode in split) E="";; nosplit) E="LGS_NO_CU_SPLIT=1";; sets3) E="LGS_LIB=$H LGS_PIPE_SETS=3";; esac
  env $E timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06bf_trace_$mode -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 --no-cpu --wl-steps 0 > gpurun_out/r06bf_bench_$mode.log 2>&1 || { tail -20 gpurun_out/r06bf_bench_$mode.log; exit 1; }
  f=$(find gpurun_out/r06bf_trace_$mode -name "*kernel_trace.csv" | head -1)
  echo "== $mode" | tee -a gpurun_out/r06bf_timeline.log
  python3 tools/trace_timeline.py $f 3 | tee -a gpurun_out/r06bf_timeline.log
  rm -rf gpurun_out/r06bf_trace_$mode
done
L=gpurun_out/r06bf_bench_sets.log
: > $L
for rep in 1 2; do for mode in split sets3; do
  case $mode in split) E="";; sets3) E="LGS_LIB=$H LGS_PIPE_SETS=3";; esac
  echo "== $mode" >> $L
  env $E timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'cus': k.get('klein_stream_cus'), 'parity': d.get('parity_check')[:40]}))" >> $L || exit 1
done; done
cat $L
