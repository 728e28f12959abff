# round 5, first box: DS address WAR probe (the dbg1 hazard), dbg1 vs main output
# hashes, the GPU suite (state_init replay, WL tests), smoke, the default bench
# (Wang-Ling leg, reference-restatement CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
echo "== ds_war" && timeout -k 10 60 ./tools/ubench/ds_war > gpurun_out/r05a_dswar.log 2>&1; rc=$?; cat gpurun_out/r05a_dswar.log; [ $rc -eq 0 ] || exit $rc
echo "== dbg1 vs main" && LGS_LIBS=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so:$V/dbg1.so timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 65536 --reps 1 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 | tee gpurun_out/r05a_dbg1.log || exit 1
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05a_pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/r05a_pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "^E \|Error" gpurun_out/r05a_pytest_gpu.log | head -80; exit $rc; }
echo "== smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05a_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r05a_smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 400 python bench.py > gpurun_out/r05a_bench.log 2>&1; rc=$?; tail -n 1 gpurun_out/r05a_bench.log | cut -c1-3000; exit $rc
