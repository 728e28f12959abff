# round 5 final build: rocprof roofline passes of the bench command with isolated launches
# (LGS_NO_PIPE=1, tools/gpu_roofline.sh), then the default bench against the committed counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== roofline" && timeout -k 10 900 bash tools/gpu_roofline.sh r05y > gpurun_out/roof_r05y.log 2>&1; rc=$?; tail -n 2 gpurun_out/roof_r05y.log | cut -c1-300; exit $rc
