set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=lattice-gaussian-mcmc_amd/build/var
L=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
echo "== samplez tests" && timeout -k 10 600 python -m pytest tests -m gpu -x -q -k samplez > gpurun_out/pytest_sz.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_sz.log; [ $rc -eq 0 ] || { grep -B5 -A40 "^E \|Error" gpurun_out/pytest_sz.log | head -80; exit $rc; }
echo "== gpu tests" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "^E \|Error" gpurun_out/pytest_gpu.log | head -80; exit $rc; }
echo "== kbench" && LGS_DEBUG_SZC=1 LGS_LIBS=$L:$V/nosz.so timeout -k 10 300 python tools/kbench.py --reps 3 2>&1 | grep -v amdgpu.ids &&
LGS_SAMPLEZ_LIBM=1 timeout -k 10 300 python tools/kbench.py --reps 3 2>&1 | grep -v amdgpu.ids &&
echo "== bench" && timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench5.log 2>&1; rc=$?; tail -1 gpurun_out/bench5.log; exit $rc
