# Speculative sub-panels: output hashes (z, log weights) of the default build against
# the LGS_NO_SPEC build (build/var/nospec.so) in reference / Wang-Ling mode, center 0
# (speculation kept) and a center of scale 3e4 (redone); then the GPU certificate tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in "" "--wl" "--center 30000" "--wl --center 30000"; do
  KB_ARGS="--hash --reps 1 $m" VARIANTS="main nospec" bash tools/gpu_kb.sh || exit 1
done > gpurun_out/spec_check.log 2>&1
cat gpurun_out/spec_check.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_certificate.py -x -v --timeout 120 --timeout-method thread -s > gpurun_out/pytest_cert.log 2>&1; rc=$?; grep -E "PASS|FAIL|center|passed|failed" gpurun_out/pytest_cert.log | tail -20; exit $rc
