# GPU tests + smoke, kbench of the default library against variants, rocprof roofline
# passes (tools/gpu_roofline.sh TAG) and the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02q}
mkdir -p gpurun_out
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
echo "== smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$KB_VARIANTS" ]; then echo "== kbench" && VARIANTS="main $KB_VARIANTS" bash tools/gpu_kb.sh > gpurun_out/kb_$TAG.log 2>&1; rc=$?; cat gpurun_out/kb_$TAG.log; [ $rc -eq 0 ] || exit $rc; fi
echo "== roofline" && bash tools/gpu_roofline.sh $TAG > gpurun_out/roof_$TAG.log 2>&1; rc=$?; tail -n 1 gpurun_out/roof_$TAG.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1; rc=$?; tail -n 1 gpurun_out/bench_$TAG.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(json.dumps({k: j[k] for k in ('value','ms_per_step','parity_check','certificate_redos','kernel_ms')}))"; exit $rc
