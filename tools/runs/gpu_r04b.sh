set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== wl tests" && timeout -k 10 400 python -u -m pytest tests/test_gpu_wl_accept.py tests/test_gpu_certificate.py -x -v -s --timeout 300 --timeout-method thread -k "wl_accept or speculative" > gpurun_out/r04b_wl.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|scale|bounds|differ|passed|failed" gpurun_out/r04b_wl.log | tail -30; [ $rc -eq 0 ] || exit $rc
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04b_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r04b_pytest_gpu.log; exit $rc
