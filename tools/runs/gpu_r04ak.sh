# early flag check in lgs_imhk (caller's stream): stream tests, then bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== stream tests" && timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_stream.py > gpurun_out/r04ak_pytest_stream.log 2>&1; rc=$?; tail -3 gpurun_out/r04ak_pytest_stream.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
echo "== bench early" && timeout -k 10 300 python bench.py > gpurun_out/r04ak_bench_early_$i.log 2>&1 || exit $?; tail -1 gpurun_out/r04ak_bench_early_$i.log | cut -c1-160
echo "== bench sync" && LGS_NO_EARLY_CHECK=1 timeout -k 10 300 python bench.py > gpurun_out/r04ak_bench_sync_$i.log 2>&1 || exit $?; tail -1 gpurun_out/r04ak_bench_sync_$i.log | cut -c1-160
done
