# round-4 build: GPU suite, smoke, bench, roofline profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r04t}
echo "== tests" && timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== roofline profile" && timeout -k 10 900 bash tools/gpu_roofline.sh $T > gpurun_out/${T}_roof.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_roof.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'], json.dumps(d['roofline'])[:400])"; exit $rc
