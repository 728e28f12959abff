# Bench (default + T=64 variant) and rocprof trace / PMC passes of the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01g}
mkdir -p gpurun_out
echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
echo "== bench T64" && timeout -k 10 300 python bench.py --imhk-steps 64 --no-cpu > gpurun_out/bench_t64.log 2>&1; rc=$?; tail -1 gpurun_out/bench_t64.log; [ $rc -eq 0 ] || exit $rc
echo "== prof" && BENCH_ARGS="--steps 5 --warmup 2 --no-cpu" timeout -k 10 900 bash tools/gpu_prof.sh $TAG > gpurun_out/prof.log 2>&1; rc=$?; tail -3 gpurun_out/prof.log; exit $rc
