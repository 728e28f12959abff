// Micro-benchmark: fp64 MFMA 16x16x4 and fp64 VALU FMA issue rates on one wave
// per SIMD and on a full grid (device timing with hipEvents).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters, double a0) {
    d4 acc[4];
    for (int g = 0; g < 4; ++g) acc[g] = (d4){0, 0, 0, 0};
    double a = a0 + threadIdx.x, b = a0 - threadIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[g], 0, 0, 0);
    }
    double s = 0;
    for (int g = 0; g < 4; ++g) s += acc[g][0] + acc[g][1] + acc[g][2] + acc[g][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void fma_loop(double* out, int iters, double a0) {
    double x[8];
    for (int k = 0; k < 8; ++k) x[k] = a0 + k + threadIdx.x;
    const double m = 1.0000001, c = 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = fma(x[k], m, c);
    }
    double s = 0;
    for (int k = 0; k < 8; ++k) s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    double* out;
    hipMalloc(&out, sizeof(double) * 256 * 8192);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int iters = 4096;
    for (int blocks : {256, 1024, 2048, 4096}) {
        mfma_loop<<<blocks, 256>>>(out, 16, 1.0);
        hipEventRecord(a);
        mfma_loop<<<blocks, 256>>>(out, iters, 1.0);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        double flops = (double)blocks * 4 * iters * 4 * 2048.0;  // waves * iters * 4 mfma * 2*16*16*4
        printf("mfma_f64_16x16x4: blocks %d  %.3f ms  %.1f TFLOP/s\n", blocks, ms, flops / ms / 1e9);
        fma_loop<<<blocks, 256>>>(out, 16, 1.0);
        hipEventRecord(a);
        fma_loop<<<blocks, 256>>>(out, iters, 1.0);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        flops = (double)blocks * 256 * iters * 8 * 2.0;
        printf("v_fma_f64:        blocks %d  %.3f ms  %.1f TFLOP/s\n", blocks, ms, flops / ms / 1e9);
    }
    return 0;
}
