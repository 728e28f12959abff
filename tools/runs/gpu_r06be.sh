# round 6 final build with the CU split: GPU suite, smoke, default bench, certificate at
# scale (C3 2^24 / C4 2^22 / C5 2^18), rocprof roofline passes of the same build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r06be}
echo "build $(sha256sum lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so | cut -c1-16)" | tee gpurun_out/${TAG}_build.txt
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "^E \|Error" gpurun_out/${TAG}_pytest_gpu.log | head -80; exit $rc; }
echo "== smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1; rc=$?; tail -n 1 gpurun_out/${TAG}_bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
cat gpurun_out/${TAG}_build.txt > gpurun_out/${TAG}_cert.log
for c in "C3_ntru512 16777216" "C4_qary1024 4194304" "C5_ntru2048 262144"; do set -- $c
  echo "== cert $1 $2" && timeout -k 10 400 python -u tools/cert_mismatch.py --config $1 --total $2 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-400 | tee -a gpurun_out/${TAG}_cert.log || exit 1
done
echo "== roofline" && timeout -k 10 1200 bash tools/gpu_roofline.sh ${TAG}r > gpurun_out/${TAG}_roof.log 2>&1; rc=$?; tail -n 3 gpurun_out/${TAG}_roof.log | cut -c1-300; exit $rc
