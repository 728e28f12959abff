# Klein probes + B z A/B: kbench of library variants (build/var/<name>.so; "main" = default lib)
#   KVARS="main v1 ..." BZVARS="main v2 ..." bash tools/gpu_probe.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-probe}
mkdir -p gpurun_out
if [ -n "$KVARS" ]; then VARIANTS="$KVARS" bash tools/gpu_kb.sh > gpurun_out/${TAG}_klein.log 2>&1 || { cat gpurun_out/${TAG}_klein.log; exit 1; }; cat gpurun_out/${TAG}_klein.log; fi
if [ -n "$BZVARS" ]; then VARIANTS="$BZVARS" KB_ARGS="--bz" bash tools/gpu_kb.sh > gpurun_out/${TAG}_bz.log 2>&1 || { cat gpurun_out/${TAG}_bz.log; exit 1; }; cat gpurun_out/${TAG}_bz.log; fi
