set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log &&
echo "== gpu tests" && timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench1.log 2>&1; rc=$?; tail -5 gpurun_out/bench1.log; exit $rc
