set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
V=lattice-gaussian-mcmc_amd/build/var
echo "== gpu tests" && timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "^E \|Error" gpurun_out/pytest_gpu.log | head -60; exit $rc; }
for cfg in "32 2 $L" "32 2 $V/lb3.so" "16 2 $L" "32 4 $L" "16 4 $L"; do
  set -- $cfg
  echo "panel=$1 zint=$2 lib=$3"
  LGS_PANEL=$1 LGS_ZINT=$2 LGS_LIBS=$3 timeout -k 10 300 python tools/kbench.py --reps 3 2>&1 | grep -v amdgpu.ids || exit 1
done
