# round 6: the default CU split (product library): stream tests, then bench A/B
# (default vs LGS_NO_CU_SPLIT=1, alternating) at C3 x2, C4, C5, C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== stream tests" && timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06bc_pytest_stream.log 2>&1; rc=$?; tail -1 gpurun_out/r06bc_pytest_stream.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/r06bc_pytest_stream.log; exit $rc; }
L=gpurun_out/r06bc_bench_cusplit_ab.log
: > $L
for cfg in C3_ntru512 C3_ntru512 C4_qary1024 C5_ntru2048 C2_qary128; do for ns in 0 1; do
  echo "== $cfg no_cu_split=$ns" >> $L
  LGS_NO_CU_SPLIT=$ns timeout -k 10 300 python bench.py --config $cfg --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'cus': k.get('klein_stream_cus'), 'parity': d.get('parity_check')[:40]}))" >> $L || exit 1
done; done
cat $L
