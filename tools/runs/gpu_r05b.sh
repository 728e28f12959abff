# round 5: GPU suite + smoke + bench of the state_init / WL-leg build; Klein A/B:
# three-address near-field FMAs (fmaasm) vs main; the round-4 dbg1 hazard with the
# round-4 Philox form (v_mad_u64_u32: dbg1m vs basem)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
M=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
echo "== kbench C3" && for r in 1 2; do LGS_LIBS=$M:$V/fmaasm.so timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1; done | tee gpurun_out/r05b_kb.log
echo "== hazard repro" && LGS_LIBS=$V/basem.so:$V/dbg1m.so timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 65536 --reps 1 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 | tee gpurun_out/r05b_dbg1m.log || exit 1
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05b_pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/r05b_pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "^E \|Error" gpurun_out/r05b_pytest_gpu.log | head -80; exit $rc; }
echo "== smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05b_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r05b_smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 400 python bench.py > gpurun_out/r05b_bench.log 2>&1; rc=$?; tail -n 1 gpurun_out/r05b_bench.log | cut -c1-4000; exit $rc
