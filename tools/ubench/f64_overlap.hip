// Do fp64 MFMA and fp64 VALU FMA from different waves of one SIMD overlap?
// mode 0: all waves MFMA, 1: all waves VALU FMA, 2: even waves MFMA / odd waves FMA,
// 3: VALU exp-heavy (transcendental) waves, 4: even MFMA / odd exp-heavy.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

__device__ double mfma_work(int iters, double a, double b) {
    d4 acc[4];
    for (int g = 0; g < 4; ++g) acc[g] = (d4){0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[g], 0, 0, 0);
    }
    double s = 0;
    for (int g = 0; g < 4; ++g) s += acc[g][0] + acc[g][1] + acc[g][2] + acc[g][3];
    return s;
}
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v4o __attribute__((ext_vector_type(4)));
__device__ double i8_work(int iters, int seed) {
    v4o acc[8];
    for (int g = 0; g < 8; ++g) acc[g] = (v4o){0, 0, 0, 0};
    v4i x = {seed, seed * 3, seed * 5, seed * 7}, y = {seed + 1, seed + 2, seed + 3, seed + 4};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int g = 0; g < 8; ++g) acc[g] = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, y, acc[g], 0, 0, 0);
    }
    int s = 0;
    for (int g = 0; g < 8; ++g) s += acc[g][0] + acc[g][1] + acc[g][2] + acc[g][3];
    return (double)s;
}
__device__ double fma_work(int iters, double a) {
    double x[8];
    for (int k = 0; k < 8; ++k) x[k] = a + k;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = fma(x[k], 1.0000001, 1e-9);
    }
    double s = 0;
    for (int k = 0; k < 8; ++k) s += x[k];
    return s;
}
__device__ double exp_work(int iters, double a) {
    double x = a * 1e-3, s = 0;
    for (int it = 0; it < iters; ++it) {
        s += exp(-x * x);
        x += 1e-7;
    }
    return s;
}
__global__ __launch_bounds__(256) void k(double* out, int mode, int im, int iv, int ie) {
    const int w = threadIdx.x >> 6;
    double a = 1.0 + threadIdx.x * 1e-3, r;
    bool m = (mode == 0) || ((mode == 2 || mode == 4) && (w & 1) == 0);
    bool q = (mode == 5) || ((mode == 6 || mode == 7) && (w & 1) == 0);
    if (q) r = i8_work(im * 4, threadIdx.x);
    else if (m) r = mfma_work(im, a, 2.0 - a);
    else if (mode == 1 || mode == 2 || mode == 6) r = fma_work(iv, a);
    else r = exp_work(ie, a);
    out[blockIdx.x * 256 + threadIdx.x] = r;
}
int main() {
    double* out;
    (void)hipMalloc(&out, sizeof(double) * 256 * 4096);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int blocks = 2048, im = 1024, iv = 4096 * 4, ie = 4096;
    for (int mode = 0; mode < 8; ++mode) {
        k<<<blocks, 256>>>(out, mode, 4, 16, 16);
        (void)hipEventRecord(a);
        k<<<blocks, 256>>>(out, mode, im, iv, ie);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("mode %d: %.3f ms\n", mode, ms);
    }
    return 0;
}
