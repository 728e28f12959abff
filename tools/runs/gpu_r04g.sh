# bench + roofline profile of the current build; Klein A/B against round 3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r04g}
[ -n "$SKIPBENCH" ] || { echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline'].get('counters'))"; [ $rc -eq 0 ] || exit $rc; }
V=lattice-gaussian-mcmc_amd/build/var
echo "== kbench A/B" && for r in 1 2; do LGS_LIBS=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so:$V/r03.so timeout -k 10 400 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 --bz || exit 1; done > gpurun_out/${T}_ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/${T}_ab.log | cut -c1-220; [ $rc -eq 0 ] || exit $rc
echo "== roofline profile" && timeout -k 10 900 bash tools/gpu_roofline.sh $T > gpurun_out/${T}_roof.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_roof.log | cut -c1-600; exit $rc
