# final tree: GPU suite, smoke, bench (library build 31ad460b, profiled in r04al)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== tests" && timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/r04an_pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/r04an_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04an_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r04an_smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/r04an_bench.log 2>&1; rc=$?; tail -1 gpurun_out/r04an_bench.log | cut -c1-200; exit $rc
