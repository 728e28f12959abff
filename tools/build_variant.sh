# Builds a diagnostic / experimental variant of the HIP library (CPU, cross-compiled):
#   bash tools/build_variant.sh NAME [-DFLAG ...]  ->  lattice-gaussian-mcmc_amd/build/var/NAME.so
# (bench.py / tools/kbench.py load it with LGS_LIB / LGS_LIBS)
set -e
cd "$(dirname "$0")/../lattice-gaussian-mcmc_amd"
name=$1; shift
mkdir -p build/var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-pass-failed \
  -mllvm -pragma-unroll-threshold=200000 -mllvm -amdgpu-use-amdgpu-trackers=1 -mllvm -amdgpu-schedule-metric-bias=50 \
  -DLGS_TEST_HOOKS "$@" -shared -o build/var/$name.so \
  csrc/lgs_kernels.hip csrc/lgs_diag.hip csrc/lgs_capi.hip
echo built build/var/$name.so
