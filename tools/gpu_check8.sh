set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== oz tests" && timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "int8_digit or goldens or ntru1024" > gpurun_out/pytest_oz.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_oz.log; [ $rc -eq 0 ] || { grep -B5 -A40 "^E \|Error" gpurun_out/pytest_oz.log | head -80; exit $rc; }
echo "== gpu tests" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "^E \|Error" gpurun_out/pytest_gpu.log | head -80; exit $rc; }
VARIANTS="main nosz nofar" bash tools/gpu_kb.sh &&
LGS_FAR=fp64 VARIANTS="main" bash tools/gpu_kb.sh &&
echo "== bench" && timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench8.log 2>&1; rc=$?; tail -1 gpurun_out/bench8.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['kernel_ms'])"; exit $rc
