# functionals of the leading chains: stream tests, then the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== tests" && timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stream.py > gpurun_out/r04j_t.log 2>&1; rc=$?; tail -3 gpurun_out/r04j_t.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/r04j_bench.log 2>&1 || { tail -5 gpurun_out/r04j_bench.log; exit 1; }
tail -1 gpurun_out/r04j_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline'].get('counters'), d['roofline'].get('frac'))"
