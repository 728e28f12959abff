# kbench over library variants: VARIANTS="name ..." (build/var/<name>.so; "main" = default lib)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=""
for v in ${VARIANTS:-main}; do
  if [ $v = main ]; then f=lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so; else f=lattice-gaussian-mcmc_amd/build/var/$v.so; fi
  L="$L:$f"
done
LGS_LIBS=${L#:} timeout -k 10 600 python tools/kbench.py --reps 3 ${KB_ARGS} 2>&1 | grep -v amdgpu.ids
