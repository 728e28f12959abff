# B z A/B with output hashes (z, log weights, v) of library variants: VARIANTS="main v ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in C3_ntru512 C4_qary1024; do
  KB_ARGS="--bz --hash --config $cfg" bash tools/gpu_kb.sh || exit 1
done
