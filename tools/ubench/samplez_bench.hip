// Micro-benchmark: cost of one SampleZ draw per lane, by path, at Klein-like
// occupancy.  Each lane draws NC coordinates with wave-uniform sigma (as in the
// sampler: all lanes of a wave are on the same coordinate) and per-lane mean.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../lattice-gaussian-mcmc_amd/csrc samplez_bench.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "lgs_device.h"
#include "lgs_szc_host.h"

using namespace lgs;

__constant__ double* szc;

__device__ __noinline__ double trivial_call(double mu, double u, const double* q) {
    return rint(mu + u * 1e-300) + q[0] * 0.0;
}

template <int MODE>
__global__ __launch_bounds__(256) void sz_kernel(const double* __restrict__ sigs, int nc,
                                                 const double* __restrict__ etab, double* out) {
    __shared__ double tab_lds[2 * (kErfTabLast + 1)];
    if (MODE == 4) {
        for (int k = threadIdx.x; k < 2 * (kErfTabLast + 1); k += blockDim.x) tab_lds[k] = etab[k];
        __syncthreads();
    }
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    CoordStream rs;
    rs.init(12345, 0, (uint32_t)p);
    double acc = 0.0;
    for (int i = 0; i < nc; ++i) {
        const double u = rs.u((uint32_t)i);
        const double v = rs.u((uint32_t)(i + nc + (i & 1)));  // per-lane mean
        const double mu = (v - 0.5) * 2000.0;
        const double s = sigs[i];
        int64_t z;
        if (MODE == 0) z = (int64_t)rint(mu + u * 1e-300);
        else if (MODE == 5) z = (int64_t)trivial_call(mu, u, sigs + i);
        else if (MODE == 1) z = sample_z(mu, s, 10, false, u, false, etab).z;
        else if (MODE == 2) z = sample_z(mu, s, 10, false, u, false, nullptr).z;
        else if (MODE == 3) {
            double ln;
            z = (int64_t)sample_z_coord(mu, u, cst(szc) + (size_t)i * kSzcStride, 10, false, false, etab, ln);
        } else {
            double ln;
            z = (int64_t)sample_z_coord(mu, u, cst(szc) + (size_t)i * kSzcStride, 10, false, false,
                                        (lds_cdptr)tab_lds, ln);
        }
        acc += (double)z;
    }
    out[p] = acc;
}

int main() {
    const int nc = 256, lanes = 1 << 18;
    double *sig_w, *sig_s, *out, *etab;
    hipMalloc(&sig_w, nc * 8);
    hipMalloc(&sig_s, nc * 8);
    hipMalloc(&out, lanes * 8);
    std::vector<double> hw(nc), hs(nc), tab(2 * (kErfTabLast + 1));
    for (int i = 0; i < nc; ++i) {
        hw[i] = 50.0 * std::pow(2176.0 / 50.0, (double)i / (nc - 1));
        hs[i] = 1.0e-3 + 2e-3 * (double)i / nc;
    }
    for (int j = 0; j <= kErfTabLast; ++j) {
        long double y = (long double)j / 64.0L;
        tab[2 * j] = (double)erfl(y);
        tab[2 * j + 1] = (double)expl(-y * y);
    }
    hipMalloc(&etab, tab.size() * 8);
    hipMemcpy(etab, tab.data(), tab.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(sig_w, hw.data(), nc * 8, hipMemcpyHostToDevice);
    hipMemcpy(sig_s, hs.data(), nc * 8, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int occ_lds = 0;
    auto run = [&](const char* name, auto kern, const double* sg) {
        kern<<<lanes / 256, 256, occ_lds>>>(sg, nc, etab, out);
        hipEventRecord(a);
        for (int r = 0; r < 3; ++r) kern<<<lanes / 256, 256, occ_lds>>>(sg, nc, etab, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= 3;
        const double draws = (double)lanes * nc;
        // SIMD-cycles per wave-draw at 2.4 GHz, 1024 SIMDs
        printf("%-24s %8.3f ms  %7.3f ns/draw(total)  %7.0f SIMD-cycles/wave-draw\n", name, ms,
               ms * 1e6 / draws, ms * 1e-3 * 2.4e9 * 1024 / (draws / 64));
    };
    std::vector<double> q(2 * nc * kSzcStride, 0.0);
    for (int i = 0; i < nc; ++i) {
        lgs_host::build_szc(hw[i], 10, q.data() + (size_t)i * kSzcStride);
        lgs_host::build_szc(hs[i], 10, q.data() + ((size_t)nc + i) * kSzcStride);
    }
    double* dq;
    hipMalloc(&dq, q.size() * 8);
    hipMemcpy(dq, q.data(), q.size() * 8, hipMemcpyHostToDevice);
    for (int occ : {8, 4, 2, 1}) {
        occ_lds = occ == 8 ? 0 : (160 * 1024) / occ - 1024;
        if (occ_lds > 65536) occ_lds = 65536 + 1024;  // probe; may fail
        double* qw = dq;
        printf("--- waves/SIMD <= %d (dynamic LDS %d B)\n", occ, occ_lds);
        hipMemcpyToSymbol(HIP_SYMBOL(szc), &qw, sizeof(qw));
        run("philox+round (wide)", sz_kernel<0>, sig_w);
        run("philox+trivial call", sz_kernel<5>, sig_w);
        run("wide  tab", sz_kernel<1>, sig_w);
        run("wide  libm", sz_kernel<2>, sig_w);
        run("wide  coord", sz_kernel<3>, sig_w);
        run("wide  coord lds", sz_kernel<4>, sig_w);
        qw = dq + (size_t)nc * kSzcStride;
        hipMemcpyToSymbol(HIP_SYMBOL(szc), &qw, sizeof(qw));
        run("small tab", sz_kernel<1>, sig_s);
        run("small coord", sz_kernel<3>, sig_s);
        run("small coord lds", sz_kernel<4>, sig_s);
        printf("    last error: %s\n", hipGetErrorString(hipGetLastError()));
    }
    return 0;
}
