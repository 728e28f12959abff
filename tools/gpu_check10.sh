set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== gpu tests" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "^E \|Error" gpurun_out/pytest_gpu.log | head -80; exit $rc; }
echo "== gpu tests fp64 far" && LGS_FAR=fp64 timeout -k 10 900 python -m pytest tests -m gpu -x -q -k "klein or imhk" > gpurun_out/pytest_gpu64.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_gpu64.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench10.log 2>&1; rc=$?; tail -1 gpurun_out/bench10.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['kernel_ms'])"; exit $rc
