# round 5: where the bench's B z time goes -- the same bench with the ||v||^2 rows
# dropped (LGS_DIAG_BZ=1), the selections dropped (2), both (3); timing probes only
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r05j
for r in 1 2; do for m in 0 1 2 3; do
  echo "== LGS_DIAG_BZ=$m"
  LGS_DIAG_BZ=$m timeout -k 10 300 python bench.py --no-cpu --wl-steps 0 --steps 8 > gpurun_out/${TAG}_b$m.log 2>&1 || { tail -20 gpurun_out/${TAG}_b$m.log; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/${TAG}_b$m.log') if x.startswith('{')][-1]; j=json.loads(l); print($m, j['value'], j['ms_per_step'], j['kernel_ms'])"
done; done | tee gpurun_out/${TAG}_bz_probe.log
echo "== overlap probe" && timeout -k 10 300 python tools/overlap_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${TAG}_overlap_probe.log
