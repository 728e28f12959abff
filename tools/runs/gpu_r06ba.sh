# round 6: the Klein stream's queue masked off k CUs (LGS_PIPE_CU_RESERVE, hooks build
# cumask.so) so the previous block's B z runs beside the Klein launch; pipelined bench,
# k = 0 / 16 / 32 / 48 / 64, spread (pat 0) and top-index (pat 1) masks, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06ba_bench_cumask.log
: > $L
for rep in 1 2; do for cfg in "0 0" "16 0" "32 0" "48 0" "64 0" "32 1" "64 1"; do
  set -- $cfg
  echo "== reserve $1 pat $2" >> $L
  LGS_PIPE_CU_RESERVE=$1 LGS_PIPE_CU_PAT=$2 LGS_LIB=$V/cumask.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'parity': d.get('parity_check')[:40]}))" >> $L || exit 1
done; done
cat $L
