# final round-4 build: per-config throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== bench_configs" && timeout -k 10 600 python -u tools/bench_configs.py 2>&1 | grep -v amdgpu.ids | cut -c1-400
