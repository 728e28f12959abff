# round 5: the stream / IMHK / parity tests under each pipelining switch (one GPU
# process per mode): every combination must give the same outputs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05z}
: > gpurun_out/${TAG}_modes.log
for mode in "LGS_NO_PIPE=1" "LGS_NO_LOOKAHEAD=1" "LGS_LOOKAHEAD_EARLY=1" "LGS_PIPE_SETS=3" "LGS_NO_BZ_MOMENTS=1" "LGS_PIPE_PRIO=1" "LGS_NO_EARLY_CHECK=1"; do
  echo "== $mode" | tee -a gpurun_out/${TAG}_modes.log
  env $mode timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_imhk_step.py tests/test_gpu_rccl.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_mode.log 2>&1; rc=$?
  tail -1 gpurun_out/${TAG}_mode.log | tee -a gpurun_out/${TAG}_modes.log
  [ $rc -eq 0 ] || { grep -B5 -A30 "^E \|Error" gpurun_out/${TAG}_mode.log | head -60; exit $rc; }
done
echo "== bench" && timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1; rc=$?; tail -n 1 gpurun_out/${TAG}_bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; l=[x for x in open('gpurun_out/${TAG}_bench.log') if x.startswith('{')][-1]; j=json.loads(l); r=j['roofline']; print({k: r.get(k) for k in ('achieved','frac','kernel_ms_avg','kernel_ms_rocprof','counters','traffic','profile_env')})"
