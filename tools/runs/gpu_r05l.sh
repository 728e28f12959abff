# round 5: pipelined blocks with the Klein stream at the lowest priority (the previous
# block's dependants dispatched first) against the default priority and no pipelining;
# the stream tests (pipelined multi-call equality)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r05l
hipcc --offload-arch=gfx950 -o /tmp/prio tools/ubench/stream_prio.cpp 2>/dev/null && /tmp/prio || true
echo "== stream tests" && timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_stream.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_pytest_stream.log; [ $rc -eq 0 ] || { grep -B5 -A30 "^E \|Error" gpurun_out/${TAG}_pytest_stream.log | head -80; exit $rc; }
for r in 1 2; do for m in "LGS_NO_PIPE=1" "LGS_PIPE_PRIO=0" "LGS_PIPE_PRIO=2"; do
  echo "== $m"
  env $m timeout -k 10 300 python bench.py --no-cpu --wl-steps 0 --steps 10 > gpurun_out/${TAG}_b.log 2>&1 || { tail -20 gpurun_out/${TAG}_b.log; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/${TAG}_b.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernel_ms']; print('$m', j['value'], j['ms_per_step'], {x: k[x] for x in ('klein','bz','accept','moments')}, j['parity_check'])"
done; done | tee gpurun_out/${TAG}_bench_ab.log
