set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== oz tests" && timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "int8_digit" > gpurun_out/pytest_oz.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_oz.log; [ $rc -eq 0 ] || { grep -B5 -A40 "^E \|Error" gpurun_out/pytest_oz.log | head -80; exit $rc; }
echo "== oz goldens" && LGS_FAR=int8 timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "goldens or ntru1024 or oracle_seeded or imhk" > gpurun_out/pytest_oz2.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_oz2.log; [ $rc -eq 0 ] || { grep -B5 -A40 "^E \|Error" gpurun_out/pytest_oz2.log | head -80; exit $rc; }
VARIANTS="main" bash tools/gpu_kb.sh && LGS_FAR=int8 VARIANTS="main" bash tools/gpu_kb.sh
