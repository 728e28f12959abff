// Dependent-latency probes for the Klein near-field model (cycles per dependent step,
// one wave per SIMD and two): fp64 FMA chain, fp64 chain with a wave-uniform branch
// per step, 22 broadcast ds_read_b128 of one record then a use, v_mad_u64_u32 chain.
// hipcc --offload-arch=gfx950 -O3 -o /tmp/latency tools/ubench/latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void fma_chain(double* out, int iters) {
    double x = 1.0 + threadIdx.x * 1e-3;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 64; ++c) x = fma(x, 0.9999999, 1e-9);
    }
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

__global__ __launch_bounds__(256) void fma_branch_chain(double* out, int iters) {
    double x = 1.0 + threadIdx.x * 1e-3;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            x = fma(x, 0.9999999, 1e-9);
            if (__builtin_amdgcn_readfirstlane(x > 100.0 ? 1 : 0)) x *= 0.5;  // never taken
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

__global__ __launch_bounds__(256) void fma_ballot_chain(double* out, int iters) {
    double x = 1.0 + threadIdx.x * 1e-3;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            x = fma(x, 0.9999999, 1e-9);
            if (__builtin_amdgcn_ballot_w64(x > 100.0) != 0) x *= 0.5;  // never taken
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

__global__ __launch_bounds__(256) void fma_exec_chain(double* out, int iters) {
    double x = 1.0 + threadIdx.x * 1e-3;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            x = fma(x, 0.9999999, 1e-9);
            if (x > 100.0) x = sqrt(x) * 0.5;  // never taken: a divergent if (saveexec + execz)
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

__global__ __launch_bounds__(256) void fma_select_chain(double* out, int iters) {
    double x = 1.0 + threadIdx.x * 1e-3;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            x = fma(x, 0.9999999, 1e-9);
            x = x > 100.0 ? x * 0.5 : x;  // a select: no branch
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

__global__ __launch_bounds__(256) void lds_record(double* out, int iters) {
    typedef double d2v __attribute__((ext_vector_type(2)));
    __shared__ d2v rec[64 * 22];
    for (int e = threadIdx.x; e < 64 * 22; e += 256) rec[e] = (d2v){e * 1e-3, 1.0};
    __syncthreads();
    double x = threadIdx.x * 1e-9;
    for (int it = 0; it < iters; ++it) {
        // the record index depends on x (as the next coordinate's record follows its z)
        const int r = __builtin_amdgcn_readfirstlane((int)(x * 1e-30)) + (it & 63);
        const d2v* p = rec + r * 22;
        d2v v[22];
#pragma unroll
        for (int k = 0; k < 22; ++k) v[k] = p[k];
#pragma unroll
        for (int k = 0; k < 22; ++k) asm volatile("" : "+v"(v[k]));
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 22; ++k) s += v[k][0] * v[k][1];
        x = fma(x, 1e-3, s * 1e-20);
    }
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

__global__ __launch_bounds__(256) void mad64_chain(double* out, int iters) {
    unsigned c0 = threadIdx.x, c1 = 7;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 32; ++c) {
            const unsigned long long m = (unsigned long long)0xD2511F53u * c0;
            c0 = (unsigned)(m >> 32) ^ c1;
            c1 = (unsigned)m;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0 + c1;
}

int main() {
    double* out;
    (void)hipMalloc(&out, sizeof(double) * 256 * 1024);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    int dev = 0;
    hipDeviceProp_t pr;
    (void)hipGetDeviceProperties(&pr, dev);
    const double ghz = pr.clockRate * 1e-6;
    const int cus = pr.multiProcessorCount;
    auto run = [&](const char* nm, auto kern, int occ, int iters, int steps) {
        const int blocks = cus * occ;
        const int lds = occ == 1 ? 100 * 1024 : 64 * 1024;
        kern<<<blocks, 256, lds>>>(out, 4);
        (void)hipEventRecord(e0);
        kern<<<blocks, 256, lds>>>(out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-24s waves/SIMD %d: %8.3f ms = %7.1f cycles per step per wave (%s)\n", nm, occ, ms,
               ms * 1e6 * ghz / ((double)iters * steps), hipGetErrorString(hipGetLastError()));
    };
    printf("clock %.3f GHz, %d CUs\n", ghz, cus);
    for (int occ : {1, 2}) {
        run("fp64 fma chain", fma_chain, occ, 4000, 64);
        run("fp64 fma + ubranch", fma_branch_chain, occ, 4000, 16);
        run("fp64 fma + ballot br", fma_ballot_chain, occ, 4000, 16);
        run("fp64 fma + exec br", fma_exec_chain, occ, 4000, 16);
        run("fp64 fma + select", fma_select_chain, occ, 4000, 16);
        run("22 x ds_read_b128 + use", lds_record, occ, 20000, 1);
        run("mad_u64_u32 chain", mad64_chain, occ, 4000, 32);
    }
    return 0;
}
