// Can a wave's fp64 MFMAs run in the background of its own latency-bound fp64
// VALU chain (and of other waves' VALU)?  Each iteration issues NM independent
// v_mfma_f64_16x16x4 (8 accumulators) and then a dependent chain of NC fp64 FMAs.
// mode 0: MFMA only, 1: chain only, 2: both interleaved in the same wave.
// Run at 1, 2 and 3 waves/SIMD (grid-limited via dynamic LDS).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

typedef int v4i __attribute__((ext_vector_type(4)));
// int8 MFMA (16x16x64) with a dependent chain of fp64 FMAs (CT=0) or int32 ops (CT=1)
template <int MODE, int NM, int NC, int CT>
__global__ __launch_bounds__(256) void k8(double* out, int iters) {
    v4i acc[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) acc[g] = (v4i){0, 0, 0, 0};
    v4i xa = {(int)threadIdx.x, 3, 5, 7}, xb = {1, 2, 3, (int)threadIdx.x};
    double x = 1.0 + threadIdx.x * 1e-3;
    unsigned y = threadIdx.x;
    for (int it = 0; it < iters; ++it) {
        if (MODE != 1) {
#pragma unroll
            for (int m = 0; m < NM; ++m)
                acc[m & 7] = __builtin_amdgcn_mfma_i32_16x16x64_i8(xa, xb, acc[m & 7], 0, 0, 0);
        }
        if (MODE != 0) {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                if (CT == 0) x = fma(x, 0.9999999, 1e-9);
                else y = (y ^ (y >> 3)) + 0x9e3779b9u;
            }
        }
    }
    double s = x + y;
#pragma unroll
    for (int g = 0; g < 8; ++g) s += acc[g][0] + acc[g][1] + acc[g][2] + acc[g][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE, int NM, int NC>
__global__ __launch_bounds__(256) void k(double* out, int iters) {
    d4 acc[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) acc[g] = (d4){0, 0, 0, 0};
    double a = 1.0 + threadIdx.x * 1e-3, b = 2.0 - a, x = a;
    for (int it = 0; it < iters; ++it) {
        if (MODE != 1) {
#pragma unroll
            for (int m = 0; m < NM; ++m)
                acc[m & 7] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[m & 7], 0, 0, 0);
        }
        if (MODE != 0) {
#pragma unroll
            for (int c = 0; c < NC; ++c) x = fma(x, 0.9999999, 1e-9);
        }
    }
    double s = x;
#pragma unroll
    for (int g = 0; g < 8; ++g) s += acc[g][0] + acc[g][1] + acc[g][2] + acc[g][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    double* out;
    (void)hipMalloc(&out, sizeof(double) * 256 * 8192);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 2000;
    auto run = [&](const char* nm, auto kern, int occ) {
        const int blocks = 256 * occ;  // one block per CU per wave/SIMD level
        const int lds = occ == 1 ? 100 * 1024 : (occ == 2 ? 64 * 1024 : 0);
        kern<<<blocks, 256, lds>>>(out, 4);
        (void)hipEventRecord(e0);
        kern<<<blocks, 256, lds>>>(out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s waves/SIMD %d: %8.3f ms  (%s)\n", nm, occ, ms, hipGetErrorString(hipGetLastError()));
    };
    for (int occ : {1, 2, 3}) {
        run("mfma x32", k<0, 32, 64>, occ);
        run("chain x64", k<1, 32, 64>, occ);
        run("mfma x32 + chain x64", k<2, 32, 64>, occ);
        run("mfma x16", k<0, 16, 128>, occ);
        run("chain x128", k<1, 16, 128>, occ);
        run("mfma x16 + chain x128", k<2, 16, 128>, occ);
        run("i8 x64", k8<0, 64, 128, 0>, occ);
        run("i8 x64 + f64 chain x128", k8<2, 64, 128, 0>, occ);
        run("i8 x64 + i32 chain x128", k8<2, 64, 128, 1>, occ);
        run("i32 chain x128", k8<1, 64, 128, 1>, occ);
    }
    return 0;
}
