# round 5 final build: parity under every run-time switch, one GPU
# process per mode
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05ad}
: > gpurun_out/${TAG}_modes.log
K="klein or imhk or lattice or edges or drop_in or stream or rccl"
for mode in "LGS_FAR=fp64" "LGS_KERNEL=valu" "LGS_ZINT=4" "LGS_PANEL=16" "LGS_BZ_FP64=1" "LGS_SAMPLEZ_LIBM=1" "LGS_NO_PIPE=1" "LGS_NO_BZ_MOMENTS=1" "LGS_NO_LOOKAHEAD=1" "LGS_MAX_PROPOSALS=1048576"; do
  echo "== $mode" | tee -a gpurun_out/${TAG}_modes.log
  env $mode timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/${TAG}_mode.log 2>&1; rc=$?
  tail -1 gpurun_out/${TAG}_mode.log | tee -a gpurun_out/${TAG}_modes.log
  [ $rc -eq 0 ] || { grep -B5 -A30 "^E \|Error" gpurun_out/${TAG}_mode.log | head -60; exit $rc; }
done
