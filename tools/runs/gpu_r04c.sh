set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== new tests" && timeout -k 10 500 python -u -m pytest tests/test_gpu_wl_accept.py tests/test_gpu_certificate.py -x -v -s --timeout 300 --timeout-method thread -k "wl_accept or speculative or q_panel" > gpurun_out/r04c_new.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|scale|bounds|differ|passed|failed|skip|assert" gpurun_out/r04c_new.log | tail -40; [ $rc -eq 0 ] || exit $rc
echo "== kbench" && for q in 1 0 1 0; do LGS_NO_QSKIP=$q timeout -k 10 120 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 --hash || exit 1; done > gpurun_out/r04c_kbench.log 2>&1; rc=$?; cat gpurun_out/r04c_kbench.log | tail -8; [ $rc -eq 0 ] || exit $rc
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04c_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r04c_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/r04c_bench.log 2>&1; rc=$?; tail -1 gpurun_out/r04c_bench.log | cut -c1-600; exit $rc
