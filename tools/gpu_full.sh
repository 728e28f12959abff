# GPU tests, smoke, default bench (with CPU baseline), per-config bench, rocprof trace + PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01h}
mkdir -p gpurun_out
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
echo "== smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
echo "== configs" && timeout -k 10 600 python tools/bench_configs.py > gpurun_out/bench_configs.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/bench_configs.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
echo "== prof" && BENCH_ARGS="--steps 5 --warmup 2 --no-cpu" timeout -k 10 900 bash tools/gpu_prof.sh $TAG > gpurun_out/prof.log 2>&1; rc=$?; tail -2 gpurun_out/prof.log; exit $rc
