# library on the bench's work stream (no cross-stream waits): stream tests, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== stream tests" && timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_stream.py > gpurun_out/r04am_pytest_stream.log 2>&1; rc=$?; tail -3 gpurun_out/r04am_pytest_stream.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
echo "== bench work stream" && timeout -k 10 300 python bench.py > gpurun_out/r04am_bench_work_$i.log 2>&1 || exit $?; tail -1 gpurun_out/r04am_bench_work_$i.log | cut -c1-160
echo "== bench default stream" && LGS_BENCH_DEFAULT_STREAM=1 timeout -k 10 300 python bench.py > gpurun_out/r04am_bench_default_$i.log 2>&1 || exit $?; tail -1 gpurun_out/r04am_bench_default_$i.log | cut -c1-160
done
