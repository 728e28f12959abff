set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== gpu tests" && timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_gpu.log | head -80; exit $rc; }
echo "== kbench" && timeout -k 10 300 python tools/kbench.py --reps 3 2>&1 | grep -v amdgpu.ids &&
echo "== bench" && timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench2.log 2>&1; rc=$?; tail -1 gpurun_out/bench2.log; exit $rc
