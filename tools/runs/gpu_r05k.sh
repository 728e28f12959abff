# round 5: pipelined IMHK blocks (each block's Klein launch on a high-priority stream
# into alternating buffer sets, beside the previous block's dependants) -- GPU suite,
# bench A/B against LGS_NO_PIPE=1 and the default-priority stream, overlap probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r05k
echo "== gpu tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "^E \|Error" gpurun_out/${TAG}_pytest_gpu.log | head -80; exit $rc; }
for r in 1 2; do for m in "LGS_NO_PIPE=1" "LGS_NO_PIPE=0" "LGS_PIPE_PRIO=0"; do
  echo "== $m"
  env $m timeout -k 10 300 python bench.py --no-cpu --wl-steps 0 --steps 10 > gpurun_out/${TAG}_b.log 2>&1 || { tail -20 gpurun_out/${TAG}_b.log; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/${TAG}_b.log') if x.startswith('{')][-1]; j=json.loads(l); print('$m', j['value'], j['ms_per_step'], j['kernel_ms'], j['parity_check'])"
done; done | tee gpurun_out/${TAG}_bench_ab.log
echo "== overlap probe" && timeout -k 10 300 python tools/overlap_probe.py --prio 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${TAG}_overlap_probe.log
