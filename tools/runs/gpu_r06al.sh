# round 6: the all-capped sub-panel copy of the decision (LGS_CAP_SP) under the scheduler
# flags, alone and with the decision-first record (LGS_REC_L2): kbench hashes C3 / C4 / C5
# (and Wang-Ling C3) against the product's sources, then the pipelined bench, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06al_capsp.log
: > $L
S=$V/mainhooks.so:$V/v_capsp.so:$V/v_capsp_recl2.so:$V/v_recl2.so
for c in "C3_ntru512 1048576" "C4_qary1024 1048576" "C5_ntru2048 131072"; do set -- $c
  echo "== kbench $1" >> $L
  LGS_LIBS=$S timeout -k 10 300 python tools/kbench.py --config $1 --n $2 --reps 3 --hash 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
echo "== kbench C3 wl" >> $L
LGS_LIBS=$S timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 3 --hash --wl 2>&1 | grep -v amdgpu.ids >> $L || exit 1
for rep in 1 2; do for v in mainhooks v_capsp v_capsp_recl2 v_recl2; do
  echo "== bench $v" >> $L
  LGS_LIB=$V/$v.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'parity': d.get('parity_check')[:40]}))" >> $L || exit 1
done; done
cat $L
