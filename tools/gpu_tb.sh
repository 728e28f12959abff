# GPU tests, smoke and the default bench (no rocprof).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
echo "== smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(json.dumps({k: j[k] for k in ('value','ms_per_step','parity_check','certificate_redos','kernel_ms')}))"; exit $rc
