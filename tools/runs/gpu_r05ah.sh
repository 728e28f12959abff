# round 5: B z with 64-coordinate workgroup tiles (LGS_BZ_BN=64: 106 VGPRs, four
# workgroups per CU; OCC=5: five) -- stream tests on the variant, bench A/B (isolated
# launches and the default pipelined bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=lattice-gaussian-mcmc_amd/build/var
M=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so
TAG=r05ah
echo "== stream tests bn64" && LGS_LIB=$V/bn64.so timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || { grep -B5 -A30 "^E \|Error" gpurun_out/${TAG}_pytest.log | head -60; exit $rc; }
for r in 1 2; do for lib in $M $V/bn64.so $V/bn64o5.so; do for p in 1 0; do
  echo "== $lib LGS_NO_PIPE=$p"
  LGS_LIB=$lib LGS_NO_PIPE=$p timeout -k 10 300 python bench.py --no-cpu --wl-steps 0 --steps 6 --warmup 2 > gpurun_out/${TAG}_b.log 2>&1 || { tail -20 gpurun_out/${TAG}_b.log; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/${TAG}_b.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernel_ms']; print('$lib $p', j['value'], j['ms_per_step'], {x: k[x] for x in ('klein','bz','accept','moments')}, j['parity_check'], j['covariance']['sum_zzT_sha256'])"
done; done; done | tee gpurun_out/${TAG}_bench_ab.log
