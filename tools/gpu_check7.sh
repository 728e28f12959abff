set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== gpu tests" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "^E \|Error" gpurun_out/pytest_gpu.log | head -80; exit $rc; }
echo "== bench" && timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench7.log 2>&1; rc=$?; tail -1 gpurun_out/bench7.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['kernel_ms'], j['roofline']['kernel_ms_avg'])"; exit $rc
