# round 6: kernel timeline of the pipelined bench with the CU split (rocprofv3 kernel
# trace, tools/trace_timeline.py), split on and off
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for ns in 0 1; do
  LGS_NO_CU_SPLIT=$ns timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06bf_trace_$ns -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 --no-cpu --wl-steps 0 > gpurun_out/r06bf_bench_$ns.log 2>&1 || { tail -20 gpurun_out/r06bf_bench_$ns.log; exit 1; }
  f=$(find gpurun_out/r06bf_trace_$ns -name "*kernel_trace.csv" | head -1)
  echo "== no_cu_split=$ns" | tee -a gpurun_out/r06bf_timeline.log
  python3 tools/trace_timeline.py $f 3 | tee -a gpurun_out/r06bf_timeline.log
  rm -rf gpurun_out/r06bf_trace_$ns
done
