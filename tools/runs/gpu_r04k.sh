# moments from the int16 history: parity tests, then the bench with / without it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== tests" && timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_statistics.py tests/test_gpu_edges.py tests/test_gpu_stream.py > gpurun_out/r04k_t.log 2>&1; rc=$?; tail -3 gpurun_out/r04k_t.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1; do
echo "== bench LGS_MOM_STORE=$m" && LGS_MOM_STORE=$m timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r04k_bench$m.log 2>&1 || { tail -5 gpurun_out/r04k_bench$m.log; exit 1; }
tail -1 gpurun_out/r04k_bench$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['parity_check'], d['covariance']['sum_zzT_sha256'])"
done
