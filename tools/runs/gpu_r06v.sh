# round 6: B z identity blocks (the I blocks of NTRU / q-ary bases added from the z digit
# tiles, no staging of B's digits) -- mainhooks (the product's sources) against noident:
# lattice points equal (kbench hashes, C3 / C4 / C5), bench isolated launches A/B, then the
# B z GPU tests on the product library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06v_bz_ident.log
: > $L
for c in "C3_ntru512 1048576" "C4_qary1024 1048576" "C5_ntru2048 65536"; do set -- $c
  echo "== hashes $1" >> $L
  LGS_LIBS=$V/noident.so:$V/mainhooks.so timeout -k 10 300 python tools/kbench.py --config $1 --n $2 --reps 2 --bz --hash 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
for rep in 1 2; do for v in noident mainhooks; do
  echo "== bench $v" >> $L
  LGS_NO_PIPE=1 LGS_LIB=$V/$v.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'klein': k['klein'], 'bz': k['bz'], 'parity': d.get('parity_check')}))" >> $L || exit 1
done; done
echo "== tests" >> $L
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_edges.py tests/test_gpu_configs.py -k "moment or bz or lattice or imhk or points" >> $L 2>&1 || exit 1
tail -3 $L
