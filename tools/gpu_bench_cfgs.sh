set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in "32 2" "32 4" "16 2"; do
  set -- $cfg
  echo "panel=$1 zint=$2"
  LGS_PANEL=$1 LGS_ZINT=$2 timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_cfg.log 2>&1 || { tail -5 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'])"
done
