set -o pipefail
cd $GRAFT_REPO_ROOT
V=lattice-gaussian-mcmc_amd/build/var
echo "== gpu tests" && timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "^E \|Error" gpurun_out/pytest_gpu.log | head -60; exit $rc; }
LGS_LIBS=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so:$V/diag_NO_SAMPLEZ.so:$V/diag_NO_FAR.so timeout -k 10 300 python tools/kbench.py --reps 3 2>&1 | grep -v amdgpu.ids
