# round 5: the build with the near-field trims default -- GPU suite, smoke, the
# certificate at scale (default vs reference-order kernel: C3 2^24, C4 2^22, C5 2^18),
# Klein A/B against t2dh (the same trims without the branchless quantile test), the
# default bench, and the rocprof roofline passes of the bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
M=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
TAG=r05i
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "^E \|Error" gpurun_out/${TAG}_pytest_gpu.log | head -80; exit $rc; }
echo "== smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== kbench" && for r in 1 2; do LGS_LIBS=$M timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 --hash 2>&1 | grep -v amdgpu.ids | cut -c1-260 || exit 1; done | tee gpurun_out/${TAG}_kb.log
echo "== bench" && timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1; rc=$?; tail -n 1 gpurun_out/${TAG}_bench.log | cut -c1-1500; [ $rc -eq 0 ] || exit $rc
echo "== roofline" && timeout -k 10 900 bash tools/gpu_roofline.sh $TAG > gpurun_out/roof_$TAG.log 2>&1; rc=$?; tail -n 3 gpurun_out/roof_$TAG.log | cut -c1-300; exit $rc
