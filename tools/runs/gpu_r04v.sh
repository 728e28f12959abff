# round-4 build: per-config throughput and the certificate at scale (default vs
# reference-order kernel, every coefficient compared)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== bench_configs" && timeout -k 10 600 python -u tools/bench_configs.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04v_bench_configs.log | cut -c1-300 || exit 1
for c in "C3_ntru512 16777216" "C4_qary1024 4194304" "C5_ntru2048 262144"; do
  set -- $c
  echo "== cert $1 $2" && timeout -k 10 400 python -u tools/cert_mismatch.py --config $1 --total $2 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04v_cert_mismatch_$1.log | cut -c1-300 || exit 1
done
echo "== configs test" && timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_configs.py 2>&1 | tail -3
