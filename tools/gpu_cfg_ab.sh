# Klein kbench A/B over configs: VARIANTS="a b ..." CFGS="C2_qary128 C3_ntru512"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in ${CFGS:-C3_ntru512}; do
  KB_ARGS="--hash --config $cfg" bash tools/gpu_kb.sh || exit 1
done
