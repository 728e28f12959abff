# Klein / IMHK parity suite under every run-time switch of INTEGRATION.md §6 (one
# GPU process per mode): all of them must give the oracle's coefficients.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
K="klein or imhk or lattice or edges or drop_in"
for mode in "LGS_FAR=fp64" "LGS_KERNEL=valu" "LGS_ZINT=4" "LGS_PANEL=16" "LGS_BZ_FP64=1" "LGS_SAMPLEZ_LIBM=1"; do
  echo "== $mode"
  env $mode timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "$K" > gpurun_out/pytest_mode.log 2>&1; rc=$?
  tail -1 gpurun_out/pytest_mode.log
  [ $rc -eq 0 ] || { grep -B5 -A30 "^E \|Error" gpurun_out/pytest_mode.log | head -60; exit $rc; }
done
