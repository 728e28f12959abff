# round 6: the Philox round keys left to loop-invariant motion (LGS_PHILOX_HOIST) against the
# product's sources: kbench hashes C3 / C4 / C5 / Wang-Ling C3, pipelined bench x3, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06an_philhoist.log
: > $L
S=$V/mainhooks.so:$V/w_philhoist.so
for c in "C3_ntru512 1048576" "C4_qary1024 1048576" "C5_ntru2048 131072"; do set -- $c
  echo "== kbench $1" >> $L
  LGS_LIBS=$S:$S timeout -k 10 300 python tools/kbench.py --config $1 --n $2 --reps 3 --hash 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
echo "== kbench C3 wl" >> $L
LGS_LIBS=$S timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 3 --hash --wl 2>&1 | grep -v amdgpu.ids >> $L || exit 1
for rep in 1 2 3; do for v in mainhooks w_philhoist; do
  echo "== bench $v" >> $L
  LGS_LIB=$V/$v.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'parity': d.get('parity_check')[:40]}))" >> $L || exit 1
done; done
cat $L
