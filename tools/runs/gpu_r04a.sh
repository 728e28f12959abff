set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== new tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu_certificate.py tests/test_gpu_stream.py -x -v -s --timeout 120 --timeout-method thread -k "low_z1 or streams or graph" > gpurun_out/r04a_new.log 2>&1; rc=$?; tail -15 gpurun_out/r04a_new.log; [ $rc -eq 0 ] || exit $rc
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04a_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r04a_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/r04a_bench.log 2>&1; rc=$?; tail -1 gpurun_out/r04a_bench.log; exit $rc
