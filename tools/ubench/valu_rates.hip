// VALU issue cost per instruction on gfx950 (MI355X), for the Klein near field's
// instruction mix: 8 independent chains per lane (enough ILP that the issue rate,
// not the dependent latency, is measured), one wave per SIMD and two.
//   v_mul_lo_u32 / v_mul_hi_u32 (Philox's products), v_mad_u64_u32 (its round-4
//   form), v_xor_b32, v_fma_f64, v_mov_b64, v_cvt_f64_u32, v_readfirstlane_b32.
// Each instruction is emitted through inline asm (no folding); cycles per
// instruction per wave = wave lifetime (s_memtime, shader clock) / instructions.
// hipcc --offload-arch=gfx950 -O3 -o tools/ubench/valu_rates tools/ubench/valu_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(X) X X X X X X X X

template <int OP>
__global__ __launch_bounds__(256) void rate(unsigned long long* cyc, unsigned* sink, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 + 11u, a5 = a0 + 13u,
             a6 = a0 ^ 17u, a7 = a0 ^ 19u;
    double d0 = a0 * 1e-3, d1 = d0 + 1, d2 = d0 + 2, d3 = d0 + 3, d4 = d0 + 4, d5 = d0 + 5, d6 = d0 + 6,
           d7 = d0 + 7;
    unsigned long long q0 = a0, q1 = a1, q2 = a2, q3 = a3;
    const unsigned k = 0xD2511F53u;
    const double m = 0.9999999, c = 1e-9;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            if constexpr (OP == 0) {  // v_mul_lo_u32
                asm volatile(REP8("v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n"
                                  "v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "s"(k));
            } else if constexpr (OP == 1) {  // v_mul_hi_u32
                asm volatile(REP8("v_mul_hi_u32 %0, %0, %8\n v_mul_hi_u32 %1, %1, %8\n v_mul_hi_u32 %2, %2, %8\n v_mul_hi_u32 %3, %3, %8\n"
                                  "v_mul_hi_u32 %4, %4, %8\n v_mul_hi_u32 %5, %5, %8\n v_mul_hi_u32 %6, %6, %8\n v_mul_hi_u32 %7, %7, %8\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "s"(k));
            } else if constexpr (OP == 2) {  // v_xor_b32
                asm volatile(REP8("v_xor_b32 %0, %8, %0\n v_xor_b32 %1, %8, %1\n v_xor_b32 %2, %8, %2\n v_xor_b32 %3, %8, %3\n"
                                  "v_xor_b32 %4, %8, %4\n v_xor_b32 %5, %8, %5\n v_xor_b32 %6, %8, %6\n v_xor_b32 %7, %8, %7\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "s"(k));
            } else if constexpr (OP == 3) {  // v_fma_f64
                asm volatile(REP8("v_fma_f64 %0, %0, %8, %9\n v_fma_f64 %1, %1, %8, %9\n v_fma_f64 %2, %2, %8, %9\n v_fma_f64 %3, %3, %8, %9\n"
                                  "v_fma_f64 %4, %4, %8, %9\n v_fma_f64 %5, %5, %8, %9\n v_fma_f64 %6, %6, %8, %9\n v_fma_f64 %7, %7, %8, %9\n")
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                             : "s"(m), "v"(c));
            } else if constexpr (OP == 4) {  // v_mad_u64_u32 (4 chains: 8 VGPRs of accumulators)
                asm volatile(REP8("v_mad_u64_u32 %0, vcc, %4, %5, %0\n v_mad_u64_u32 %1, vcc, %4, %5, %1\n"
                                  "v_mad_u64_u32 %2, vcc, %4, %5, %2\n v_mad_u64_u32 %3, vcc, %4, %5, %3\n")
                             : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3)
                             : "s"(k), "v"(a0)
                             : "vcc");
            } else if constexpr (OP == 5) {  // v_mov_b64
                asm volatile(REP8("v_mov_b64 %0, %1\n v_mov_b64 %1, %2\n v_mov_b64 %2, %3\n v_mov_b64 %3, %4\n"
                                  "v_mov_b64 %4, %5\n v_mov_b64 %5, %6\n v_mov_b64 %6, %7\n v_mov_b64 %7, %0\n")
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7));
            } else if constexpr (OP == 6) {  // v_cvt_f64_u32
                asm volatile(REP8("v_cvt_f64_u32 %0, %8\n v_cvt_f64_u32 %1, %8\n v_cvt_f64_u32 %2, %8\n v_cvt_f64_u32 %3, %8\n"
                                  "v_cvt_f64_u32 %4, %8\n v_cvt_f64_u32 %5, %8\n v_cvt_f64_u32 %6, %8\n v_cvt_f64_u32 %7, %8\n")
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                             : "v"(a0));
            } else {  // v_readfirstlane_b32 (into SGPRs, 8 per group)
                unsigned s0, s1, s2, s3, s4, s5, s6, s7;
                asm volatile(REP8("v_readfirstlane_b32 %0, %8\n v_readfirstlane_b32 %1, %9\n v_readfirstlane_b32 %2, %10\n v_readfirstlane_b32 %3, %11\n"
                                  "v_readfirstlane_b32 %4, %12\n v_readfirstlane_b32 %5, %13\n v_readfirstlane_b32 %6, %14\n v_readfirstlane_b32 %7, %15\n")
                             : "=s"(s0), "=s"(s1), "=s"(s2), "=s"(s3), "=s"(s4), "=s"(s5), "=s"(s6), "=s"(s7)
                             : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7));
                a0 += s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7;
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) atomicAdd(cyc, t1 - t0);
    sink[blockIdx.x * 256 + threadIdx.x] =
        a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (unsigned)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7) ^ (unsigned)(q0 ^ q1 ^ q2 ^ q3);
}

template <int OP>
static void run(const char* name, int per_wave_insts_per_rep, int waves_per_simd) {
    const int cus = 256, iters = 2000;
    const int blocks = cus * waves_per_simd;  // 256-thread blocks = 4 waves = one per SIMD
    unsigned long long* cyc;
    unsigned* sink;
    (void)hipMalloc(&cyc, 8);
    (void)hipMalloc(&sink, (size_t)blocks * 256 * 4);
    (void)hipMemset(cyc, 0, 8);
    hipLaunchKernelGGL(rate<OP>, dim3(blocks), dim3(256), 0, 0, cyc, sink, 10);  // warm
    (void)hipDeviceSynchronize();
    (void)hipMemset(cyc, 0, 8);
    hipLaunchKernelGGL(rate<OP>, dim3(blocks), dim3(256), 0, 0, cyc, sink, iters);
    (void)hipDeviceSynchronize();
    unsigned long long h = 0;
    (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    const double waves = blocks * 4.0;
    const double insts = (double)iters * 8 * per_wave_insts_per_rep;
    printf("%-22s waves/SIMD %d: %6.2f cycles per instruction per wave (%.2f per SIMD)\n", name, waves_per_simd,
           h / waves / insts, h / waves / insts / waves_per_simd);
    (void)hipFree(cyc);
    (void)hipFree(sink);
}

int main() {
    for (int w = 1; w <= 2; ++w) {
        run<0>("v_mul_lo_u32", 64, w);
        run<1>("v_mul_hi_u32", 64, w);
        run<2>("v_xor_b32", 64, w);
        run<3>("v_fma_f64", 64, w);
        run<4>("v_mad_u64_u32", 32, w);
        run<5>("v_mov_b64", 64, w);
        run<6>("v_cvt_f64_u32", 64, w);
        run<7>("v_readfirstlane_b32", 64, w);
    }
    return 0;
}
