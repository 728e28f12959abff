# round 6: the new stream test alone, then the rest of the GPU suite from there, smoke, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r06c}
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_statistics.py tests/test_gpu_wl_accept.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "^E \|Error" gpurun_out/${TAG}_pytest_gpu.log | head -80; exit $rc; }
echo "== smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench.log 2>&1; rc=$?; tail -n 1 gpurun_out/${TAG}_bench.log | cut -c1-400; exit $rc
