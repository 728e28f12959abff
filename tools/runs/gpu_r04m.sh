# fused lag sums + moments_h16 (2 lanes / proposal): tests, bench, kernel trace + HBM bytes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r04m
O=gpurun_out/r04m
echo "== tests" && timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_parity.py tests/test_gpu_statistics.py tests/test_gpu_edges.py > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py --no-cpu > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['parity_check'], d['autocorrelation']['z_last'][:3])"
ARGS="--steps 3 --warmup 1 --no-cpu"
echo "== trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py $ARGS > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py $ARGS > $O/fetch.log 2>&1 || { echo fetch failed; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 bench.py $ARGS > $O/write.log 2>&1 || { echo write failed; exit 1; }
echo done
