# Klein near-field loop without store waits (sum |z| from the packed history, the capped
# tolerance constant in SGPRs): full GPU suite, kbench, bench (moments RY 4 vs 8)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r04n
O=gpurun_out/r04n
echo "== kbench" && for r in 1 2; do timeout -k 10 300 python tools/kbench.py --config C3_ntru512 --n 262144 --reps 5 --bz 2>&1 | grep -v amdgpu.ids | cut -c1-250 || exit 1; done
echo "== tests" && timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for lib in lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so lattice-gaussian-mcmc_amd/build/var/mry8.so; do
echo "== bench $lib" && LGS_LIB=$lib timeout -k 10 300 python bench.py --no-cpu > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['parity_check'], d['certificate_redos'])"
done
