set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 tools/ubench/samplez_bench > gpurun_out/szb.log 2>&1; rc=$?; grep -A10 "<= 8\|<= 2" gpurun_out/szb.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_check5.sh
