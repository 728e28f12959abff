# round 6: B z experiments -- moment partials after the chunk's MFMAs (bzlate), 16-byte
# epilogue stores (bzwide), both (bzboth) against the same sources without them
# (mainhooks): lattice points equal (kbench hashes), bench isolated launches A/B, then the
# B z / moments GPU tests on the variant with both
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
L=gpurun_out/r06q_bz_ab.log
: > $L
echo "== hashes" >> $L
LGS_LIBS=$V/mainhooks.so:$V/bzwide.so:$V/bzboth.so timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 1048576 --reps 3 --bz --hash 2>&1 | grep -v amdgpu.ids >> $L || exit 1
for rep in 1 2; do for v in mainhooks bzlate bzwide bzboth; do
  echo "== $v" >> $L
  LGS_NO_PIPE=1 LGS_LIB=$V/$v.so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu --wl-steps 0 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['kernel_ms'], 'parity': d.get('parity')}))" >> $L || exit 1
done; done
echo "== tests (bzboth)" >> $L
LGS_LIB=$V/bzboth.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_edges.py -k "moment or bz or lattice or imhk" >> $L 2>&1 || exit 1
cat $L
