# rocprofv3 kernel-trace summary + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
ARGS=${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_$TAG/bench_trace.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_$TAG/pmc_fetch -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_$TAG/bench_fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_$TAG/pmc_write -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_$TAG/bench_write.log 2>&1
rc=$?
find gpurun_out/prof_$TAG -name "*.csv" | head -20
exit $rc
