# Resource usage (VGPRs, scratch, LDS, occupancy, code size) of the bench's Klein
# kernel instantiation for a set of -D flags:  bash tools/kres.sh [-DFLAG ...]
set -e
cd "$(dirname "$0")/../lattice-gaussian-mcmc_amd"
out=$(mktemp /tmp/kres.XXXX.s)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-pass-failed -w \
  -mllvm -pragma-unroll-threshold=200000 "$@" -S --cuda-device-only -o $out csrc/lgs_kernels.hip
K=${LGS_KRES_KERNEL:-_ZN3lgs17klein_mfma_kernelIsLi32ELb0ELb1ELb0EEEvNS_9KleinArgsEPKdS3_PT_}
L=$(grep -n "^$K:" $out | cut -d: -f1)
awk -v L=$L 'NR>=L' $out | awk '/^; Occupancy/{print; exit} {print}' > ${out%.s}.k.s
echo "$* :: $(grep -E '^; (NumVgprs|NumAgprs|ScratchSize|codeLenInByte|LDSByteSize|Occupancy)' ${out%.s}.k.s | sed 's/^; //' | tr '\n' ' ')  [${out%.s}.k.s]"
rm -f $out
