// DS address write-after-read probe (the "dbg1" hazard).
//
// The dbg1 Klein build drew a Philox uniform between the near-field record's 22
// ds_read_b128 (all from one address VGPR, v0) and their first use; its ISA
// reuses that address VGPR (v_mov_b32 v0, ...) four SALU instructions after the
// last ds_read_b128 issued, while the reads are still in flight, and its outputs
// were wrong and 60x slower (garbage records).  This probe checks on the hardware
// whether a VALU write of a ds_read's address VGPR, issued before the read has
// completed, can change the address the read uses.
//
// Each wave (2 blocks of 4 waves per CU, like klein_mfma_kernel) reads 22 x 16 B
// from a record in LDS through one address register, in one asm statement:
//   mode 0: s_waitcnt lgkmcnt(0), then overwrite the address register (control)
//   mode 1: overwrite the address register right after the last read, then wait
//   mode 2: overwrite it right after the FIRST read (21 reads still to issue use
//           the new value: expected garbage -- checks the probe detects a change)
// and counts the 16-byte values that differ from the record.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/ds_war tools/ubench/ds_war.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define R16(k) "ds_read_b128 %" #k ", %22 offset:" #k "*16\n"
#define OUTS(o)                                                                                         \
    "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]),        \
        "=&v"(o[7]), "=&v"(o[8]), "=&v"(o[9]), "=&v"(o[10]), "=&v"(o[11]), "=&v"(o[12]), "=&v"(o[13]), \
        "=&v"(o[14]), "=&v"(o[15]), "=&v"(o[16]), "=&v"(o[17]), "=&v"(o[18]), "=&v"(o[19]),           \
        "=&v"(o[20]), "=&v"(o[21]), "+v"(addr)

template <int MODE>
__global__ __launch_bounds__(256, 2) void ds_war(unsigned long long* err, int iters) {
    __shared__ __attribute__((aligned(16))) unsigned int rec[32 * 92];  // 32 records of 368 B
    for (int e = threadIdx.x; e < 32 * 92; e += 256) rec[e] = 0x9E3779B9u * (unsigned)(e + 1) + blockIdx.x;
    __syncthreads();
    unsigned long long bad = 0;
    for (int it = 0; it < iters; ++it) {
        const int r = (it * 7 + (threadIdx.x >> 6)) & 31;
        unsigned int addr = (unsigned int)(uintptr_t)(&rec[r * 92]);
        addr = __builtin_amdgcn_readfirstlane(addr);
        // the overwriting value: another record's address (inside the allocation: a read
        // through it returns that record's words, never faults)
        const unsigned int junk = (unsigned int)(uintptr_t)(&rec[(r ^ 16) * 92]);
        v4u o[22];
        if constexpr (MODE == 0) {
            asm volatile(R16(0) R16(1) R16(2) R16(3) R16(4) R16(5) R16(6) R16(7) R16(8) R16(9) R16(10) R16(11)
                             R16(12) R16(13) R16(14) R16(15) R16(16) R16(17) R16(18) R16(19) R16(20) R16(21)
                         "s_waitcnt lgkmcnt(0)\n"
                         "v_mov_b32 %22, %23\n"
                         : OUTS(o)
                         : "v"(junk));
        } else if constexpr (MODE == 1) {
            asm volatile(R16(0) R16(1) R16(2) R16(3) R16(4) R16(5) R16(6) R16(7) R16(8) R16(9) R16(10) R16(11)
                             R16(12) R16(13) R16(14) R16(15) R16(16) R16(17) R16(18) R16(19) R16(20) R16(21)
                         "v_mov_b32 %22, %23\n"
                         "s_waitcnt lgkmcnt(0)\n"
                         : OUTS(o)
                         : "v"(junk));
        } else {
            asm volatile(R16(0)
                         "v_mov_b32 %22, %23\n"
                         R16(1) R16(2) R16(3) R16(4) R16(5) R16(6) R16(7) R16(8) R16(9) R16(10) R16(11)
                             R16(12) R16(13) R16(14) R16(15) R16(16) R16(17) R16(18) R16(19) R16(20) R16(21)
                         "s_waitcnt lgkmcnt(0)\n"
                         : OUTS(o)
                         : "v"(junk));
        }
        const v4u* want = (const v4u*)&rec[r * 92];
#pragma unroll
        for (int k = 0; k < 22; ++k) {
            const v4u w = want[k];
            bad += (o[k][0] != w[0]) | (o[k][1] != w[1]) | (o[k][2] != w[2]) | (o[k][3] != w[3]);
        }
        __syncthreads();  // keep the waves of a block in step (the contention of the Klein kernel)
    }
    atomicAdd(err, bad);
}

template <int MODE>
static void run(unsigned long long* d_err, int blocks, int iters) {
    hipMemset(d_err, 0, 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(ds_war<MODE>, dim3(blocks), dim3(256), 0, 0, d_err, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    unsigned long long h = 0;
    hipMemcpy(&h, d_err, 8, hipMemcpyDeviceToHost);
    const double reads = (double)blocks * 256 * iters * 22;
    printf("mode %d (%s): %llu of %.0f 16-byte reads differ, %.3f ms\n", MODE,
           MODE == 0 ? "wait, then overwrite the address" : MODE == 1 ? "overwrite the address, then wait"
                                                                      : "overwrite after the first read (expect errors)",
           h, reads, ms);
}

int main() {
    unsigned long long* d_err;
    hipMalloc(&d_err, 8);
    const int blocks = 256 * 2 * 8, iters = 2000;
    run<0>(d_err, blocks, iters);
    run<1>(d_err, blocks, iters);
    run<2>(d_err, blocks, iters);
    run<1>(d_err, blocks, iters);
    run<0>(d_err, blocks, iters);
    hipFree(d_err);
    return 0;
}
