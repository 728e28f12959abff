# round 5 final build: rocprof roofline passes of the bench command, and the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== roofline" && timeout -k 10 900 bash tools/gpu_roofline.sh r05x > gpurun_out/roof_r05x.log 2>&1; rc=$?; tail -n 2 gpurun_out/roof_r05x.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05x_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r05x_smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 400 python bench.py > gpurun_out/r05x_bench.log 2>&1; rc=$?; tail -n 1 gpurun_out/r05x_bench.log | cut -c1-600; exit $rc
