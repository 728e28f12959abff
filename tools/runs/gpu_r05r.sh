# round 5 final build: rocprof roofline passes of the bench command (kernel trace + stats, SQ / TCC PMC passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== roofline" && timeout -k 10 1000 bash tools/gpu_roofline.sh r05r > gpurun_out/roof_r05r.log 2>&1; rc=$?; tail -n 3 gpurun_out/roof_r05r.log | cut -c1-300; exit $rc
