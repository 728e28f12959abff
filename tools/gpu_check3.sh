set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== gpu tests" && timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "^E \|Error" gpurun_out/pytest_gpu.log | head -80; exit $rc; }
echo "== gpu tests (valu kernel)" && LGS_KERNEL=valu timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "klein" > gpurun_out/pytest_gpu_valu.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_gpu_valu.log; [ $rc -eq 0 ] || exit $rc
echo "== kbench" && timeout -k 10 300 python tools/kbench.py --reps 3 2>&1 | grep -v amdgpu.ids &&
LGS_KERNEL=valu timeout -k 10 300 python tools/kbench.py --reps 3 2>&1 | grep -v amdgpu.ids &&
echo "== bench" && timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench3.log 2>&1; rc=$?; tail -1 gpurun_out/bench3.log; exit $rc
