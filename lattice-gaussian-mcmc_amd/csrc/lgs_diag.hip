// lgs_diag.hip -- diagnostics on the sample stream, gfx950.
//
//   series_stats_kernel  per scalar series: mean, lag-k autocovariance / ACF
//                        (mcmc_diag.py:12-33, convergence_diag.py:75-113), the
//                        Sokal-windowed integrated autocorrelation time
//                        (mcmc_diag.py:36-56, convergence_diag.py:116-145) with an
//                        early exit once the window closes, and batch means
//                        (mcmc_diag.py:79-98, 228-241; convergence_diag.py:316-345).
//   gram_planes_kernel   exact integer second moments  sum_s z z^T  and  sum_s z of
//                        coefficient vectors (empirical mean / covariance,
//                        base.py:154-160) on v_mfma_i32_32x32x32_i8 with two balanced
//                        base-256 digits per coefficient; gram_val_kernel is the exact
//                        int64 VALU replay for |z| > 32639 and the fp64 path for
//                        real-valued samples (centred on their mean, as np.cov).
//   jump_kernel          ||x_{t+1} - x_t||_2 (mcmc_diag.py:120-136).
//   tvd_* kernels        discrete marginal total-variation distance between two
//                        sample sets (convergence_diag.py:15-48, 66-72).
//
// Series layout: series s starts at (s / gsize) * gstride + (s % gsize) * sstride
// elements and advances by tstride per time step, so a row-major (n x d) sample
// matrix (one series per coordinate), a chain-major IMHK trace (chains x steps x d)
// or a coordinate-major store are all read in place.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "lgs_kernels.h"

namespace lgs {

namespace {

template <typename XT>
__device__ __forceinline__ double as_f64(XT v) {
    return (double)v;
}

// exact integer sum (long long) or fp64 sum, as the element type allows
template <typename XT>
struct SumT {
    using T = long long;
};
template <>
struct SumT<double> {
    using T = double;
};

template <typename T>
__device__ T block_sum(T v, T* sh) {  // 256 threads, fixed tree order
    const int tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) sh[tid] += sh[tid + o];
        __syncthreads();
    }
    const T r = sh[0];
    __syncthreads();
    return r;
}

}  // namespace

// ------------------------------------------------------------ per-series statistics
// One workgroup (256 threads) per series.  Lags are processed in blocks of 64
// (16 lag quads x 16 time slices per pass); the time axis is staged through LDS
// in chunks of 4096 mean-centred values (left factor) plus the lag-shifted window
// (right factor), each thread sliding a 4-lag register window along its slice:
// 2 LDS reads per 4 FMAs.  Values past the end are staged as 0, so the pair
// (t, t+k) contributes only while t + k < n, exactly the 'full' correlation.
constexpr int kAcfCH = 4096, kAcfLB = 64;

template <typename XT>
__global__ __launch_bounds__(256) void series_stats_kernel(SeriesArgs a) {
    __shared__ double Ls[kAcfCH];
    __shared__ double Rs[kAcfCH + kAcfLB];
    __shared__ double red[16][kAcfLB];
    __shared__ double gam[kAcfLB];
    __shared__ typename SumT<XT>::T sred[256];
    __shared__ int sh_stop;
    const int tid = threadIdx.x;
    const int64_t s = (int64_t)blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
    if (s >= a.n_series) return;
    const XT* x = (const XT*)a.x + (s / a.gsize) * a.gstride + (s % a.gsize) * a.sstride;
    const int64_t n = a.n, ts = a.tstride;

    // mean (np.mean: exact for integer-valued data while |sum| < 2^53)
    typename SumT<XT>::T part = 0;
    for (int64_t t = tid; t < n; t += 256) part += x[t * ts];
    const double mean = (double)block_sum(part, sred) / (double)n;
    if (tid == 0 && a.mean) a.mean[s] = mean;

    // batch means: mean of x[j*b : (j+1)*b], j < n // b
    if (a.batch > 0 && a.bmeans) {
        const int64_t nb = n / a.batch;
        for (int64_t j = tid; j < nb; j += 256) {
            typename SumT<XT>::T bs = 0;
            for (int64_t t = j * a.batch; t < (j + 1) * a.batch; ++t) bs += x[t * ts];
            a.bmeans[s * a.ld_b + j] = (double)bs / (double)a.batch;
        }
    }
    if (a.max_lag < 0) return;

    const int64_t L = a.max_lag < n - 1 ? a.max_lag : n - 1;
    const int q = tid & 15, sl = tid >> 4;
    const int tb = sl * (kAcfCH / 16);
    double c0 = 0.0, tau = 0.0;  // thread 0's running state
    int stopped = 0;
    if (tid == 0) sh_stop = 0;
    for (int64_t kb = 0; kb <= L; kb += kAcfLB) {
        double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
        for (int64_t t0 = 0; t0 < n - kb; t0 += kAcfCH) {
            __syncthreads();
            for (int i = tid; i < kAcfCH; i += 256) {
                const int64_t t = t0 + i;
                Ls[i] = t < n ? as_f64(x[t * ts]) - mean : 0.0;
            }
            for (int i = tid; i < kAcfCH + kAcfLB; i += 256) {
                const int64_t t = t0 + kb + i;
                Rs[i] = t < n ? as_f64(x[t * ts]) - mean : 0.0;
            }
            __syncthreads();
            const double* rp = Rs + tb + 4 * q;
            double w0 = rp[0], w1 = rp[1], w2 = rp[2], w3 = rp[3];
#pragma unroll 8
            for (int tt = 0; tt < kAcfCH / 16; ++tt) {
                const double yl = Ls[tb + tt];
                acc0 += yl * w0;
                acc1 += yl * w1;
                acc2 += yl * w2;
                acc3 += yl * w3;
                w0 = w1;
                w1 = w2;
                w2 = w3;
                w3 = rp[tt + 4];
            }
        }
        red[sl][4 * q + 0] = acc0;
        red[sl][4 * q + 1] = acc1;
        red[sl][4 * q + 2] = acc2;
        red[sl][4 * q + 3] = acc3;
        __syncthreads();
        if (tid < kAcfLB) {
            double g = 0.0;
            for (int j = 0; j < 16; ++j) g += red[j][tid];
            gam[tid] = g;
        }
        __syncthreads();
        const double c0b = kb == 0 ? gam[0] : 0.0;
        if (kb == 0 && tid == 0 && a.c0) a.c0[s] = c0b;
        if (tid == 0) {
            if (kb == 0) c0 = c0b;
            for (int l = 0; l < kAcfLB && kb + l <= L; ++l) {
                const int64_t k = kb + l;
                const double r = gam[l] / c0;
                if (a.acf) a.acf[s * a.ld_acf + k] = r;
                if (k >= 1 && !stopped) {  // tau_int += 2 acf[k]; stop once k >= c tau_int
                    tau += 2.0 * r;
                    if ((double)k >= a.window_c * tau) stopped = 1;
                }
            }
            sh_stop = stopped && !a.acf;
        }
        __syncthreads();
        if (sh_stop) break;
    }
    if (tid == 0 && a.tau) a.tau[s] = 1.0 + tau;
}

// ------------------------------------------------------------ exact sum z z^T
// Block tile 128 x 128 of the d x d Gram matrix (upper tile pairs only; the
// mirrored entries are written too), K = samples split over blockIdx.y in chunks of
// kc <= 32768 so the int32 digit-class sums stay exact (2 kc 2^14 < 2^31).
// 8 waves as 2 x 4, each 64 x 32 = two 32x32 MFMA tiles; K steps of 64 samples
// through LDS as balanced base-256 digit planes [coord][sample] (pitch 80 bytes).
//   z z' = 65536 h h' + 256 (h l' + l h') + l l'
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v16i_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void atomic_add_val(long long* p, long long v) {
    atomicAdd((unsigned long long*)p, (unsigned long long)v);
}
__device__ __forceinline__ void atomic_add_val(double* p, double v) { atomicAdd(p, v); }

__device__ __forceinline__ void tile_pair(int p, int nt, int& ti, int& tj) {
    int i = 0;
    while (p >= nt - i) {
        p -= nt - i;
        ++i;
    }
    ti = i;
    tj = i + p;
}

// (1) gram_pack_kernel: y = x - shift -> balanced base-256 digit planes
//     Ph / Pl [coordinate][sample] int8 (row pitch ldp = n rounded up to 64, rows
//     up to d rounded up to 128, padding zero), read once from row-major (n x d)
//     or coordinate-major (d x n) input through a 64 x 64 LDS tile.
// (2) gram_planes_kernel: block tile 128 x 128 of the upper block triangle, 8 waves
//     as 2 x 4 (64 x 32 each = two 32x32 MFMA tiles), K steps of 64 samples: the
//     next step's 16-byte plane pieces are loaded into registers right after the
//     barrier, so the loads overlap the 16 MFMAs per wave of the current step.
//     K chunks of kc <= 16384 samples per workgroup keep the int32 class sums exact
//     (2 kc 2^14 < 2^31); results are ADDED with 64-bit atomics.
// (3) gram_mirror_kernel copies the upper block triangle into the lower one.
template <typename ZT, bool CM>
__global__ __launch_bounds__(256) void gram_pack_kernel(const ZT* __restrict__ X, int64_t ldx, int d,
                                                        int64_t n, const long long* __restrict__ shift,
                                                        int8_t* __restrict__ Ph, int8_t* __restrict__ Pl,
                                                        int64_t ldp, unsigned int* flags) {
    __shared__ int tile[64][65];  // [coordinate][sample]
    const int tid = threadIdx.x;
    const int64_t s0 = (int64_t)blockIdx.x * 64;
    const int c0 = blockIdx.y * 64;
    bool bad = false;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        // coalesced along the contiguous axis of the input
        const int fast = tid & 63, slow = e * 4 + (tid >> 6);
        const int cc = CM ? slow : fast, ss = CM ? fast : slow;
        const int c = c0 + cc;
        const int64_t s = s0 + ss;
        long long y = 0;
        if (c < d && s < n) {
            y = CM ? (long long)X[(size_t)c * ldx + s] : (long long)X[(size_t)s * ldx + c];
            if (shift) y -= shift[c];
            bad |= (y > 32639) | (y < -32639);
        }
        tile[cc][ss] = (int)y;
    }
    __syncthreads();
    const int cc = tid >> 2, part = tid & 3;
    v4i_t wl, wh;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        unsigned int lo4 = 0, hi4 = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int y = tile[cc][part * 16 + q * 4 + j];
            const int lo = (y << 24) >> 24;
            const int hi = (y - lo) >> 8;
            lo4 |= ((unsigned int)lo & 0xffu) << (8 * j);
            hi4 |= ((unsigned int)hi & 0xffu) << (8 * j);
        }
        wl[q] = (int)lo4;
        wh[q] = (int)hi4;
    }
    const size_t off = (size_t)(c0 + cc) * ldp + s0 + part * 16;
    *(v4i_t*)(Pl + off) = wl;
    *(v4i_t*)(Ph + off) = wh;
    if (bad) atomicOr(flags, kFlagI8Range);
}

__device__ __forceinline__ int digit_sum16(v4i_t h, v4i_t l) {  // sum of 256 h + l over 16 bytes
    int s = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int hb = (h[q] << (24 - 8 * j)) >> 24, lb = (l[q] << (24 - 8 * j)) >> 24;
            s += 256 * hb + lb;
        }
    return s;
}

__global__ __launch_bounds__(512) void gram_planes_kernel(const int8_t* __restrict__ Ph,
                                                          const int8_t* __restrict__ Pl, int64_t ldp,
                                                          int d, int64_t np, int64_t kc, int nt,
                                                          unsigned long long* __restrict__ G,
                                                          unsigned long long* __restrict__ S,
                                                          const unsigned int* gate) {
    // gate (nullable): the packing found a |y| beyond two digits -- the exact VALU
    // replay runs instead (decided on the device: no host round trip between the passes)
    if (gate && (*(const volatile unsigned int*)gate & kFlagI8Range)) return;
    constexpr int BT = 128, KC = 64, P = 80;
    __shared__ __attribute__((aligned(16))) int8_t A1[BT * P], A0[BT * P], B1[BT * P], B0[BT * P];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    int ti, tj;
    tile_pair((int)blockIdx.x, nt, ti, tj);
    const bool diag = ti == tj;
    const int64_t k0 = (int64_t)blockIdx.y * kc;
    const int64_t k1 = k0 + kc < np ? k0 + kc : np;
    const int row = tid >> 2, part = tid & 3;
    const int8_t* pa_h = Ph + (size_t)(ti * BT + row) * ldp + part * 16;
    const int8_t* pa_l = Pl + (size_t)(ti * BT + row) * ldp + part * 16;
    const int8_t* pb_h = Ph + (size_t)(tj * BT + row) * ldp + part * 16;
    const int8_t* pb_l = Pl + (size_t)(tj * BT + row) * ldp + part * 16;
    v16i_t h[2], m[2], l[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        h[t] = (v16i_t){};
        m[t] = (v16i_t){};
        l[t] = (v16i_t){};
    }
    int zsum = 0;
    v4i_t rah = *(const v4i_t*)(pa_h + k0), ral = *(const v4i_t*)(pa_l + k0);
    v4i_t rbh = rah, rbl = ral;
    if (!diag) {
        rbh = *(const v4i_t*)(pb_h + k0);
        rbl = *(const v4i_t*)(pb_l + k0);
    }
    const int8_t* Bh = diag ? A1 : B1;
    const int8_t* Bl = diag ? A0 : B0;
    for (int64_t k = k0; k < k1; k += KC) {
        *(v4i_t*)&A1[row * P + part * 16] = rah;
        *(v4i_t*)&A0[row * P + part * 16] = ral;
        if (!diag) {
            *(v4i_t*)&B1[row * P + part * 16] = rbh;
            *(v4i_t*)&B0[row * P + part * 16] = rbl;
        } else {
            zsum += digit_sum16(rah, ral);
        }
        __syncthreads();
        if (k + KC < k1) {  // next step's pieces in flight during the MFMAs
            rah = *(const v4i_t*)(pa_h + k + KC);
            ral = *(const v4i_t*)(pa_l + k + KC);
            if (!diag) {
                rbh = *(const v4i_t*)(pb_h + k + KC);
                rbl = *(const v4i_t*)(pb_l + k + KC);
            }
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int kb = ks * 32 + 16 * (lane >> 5);
            const int col = wn * 32 + (lane & 31);
            const v4i_t b1 = *(const v4i_t*)&Bh[col * P + kb];
            const v4i_t b0 = *(const v4i_t*)&Bl[col * P + kb];
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
                const int arow = wm * 64 + rt * 32 + (lane & 31);
                const v4i_t a1 = *(const v4i_t*)&A1[arow * P + kb];
                const v4i_t a0 = *(const v4i_t*)&A0[arow * P + kb];
                h[rt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b1, h[rt], 0, 0, 0);
                m[rt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b0, m[rt], 0, 0, 0);
                m[rt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b1, m[rt], 0, 0, 0);
                l[rt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b0, l[rt], 0, 0, 0);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int gi = ti * BT + wm * 64 + rt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
            const int gj = tj * BT + wn * 32 + (lane & 31);
            if (gi < d && gj < d) {
                const long long v = 65536LL * h[rt][reg] + 256LL * m[rt][reg] + (long long)l[rt][reg];
                if (v) atomicAdd(G + (size_t)gi * d + gj, (unsigned long long)v);
            }
        }
    if (diag && S) {  // 4 threads per row: reduce across the part lanes, one atomic per row
        zsum += __shfl_xor(zsum, 1, 64);
        zsum += __shfl_xor(zsum, 2, 64);
        const int gi = ti * BT + row;
        if (part == 0 && gi < d && zsum) atomicAdd(S + gi, (unsigned long long)(long long)zsum);
    }
}

// lower block triangle := upper (tiles ti < tj of 128); diagonal tiles are full
__global__ __launch_bounds__(256) void gram_mirror_kernel(unsigned long long* __restrict__ G, int d,
                                                          const unsigned int* gate) {
    if (gate && (*(const volatile unsigned int*)gate & kFlagI8Range)) return;
    const int j = blockIdx.x * 16 + (threadIdx.x & 15);   // column of the lower entry
    const int i = blockIdx.y * 16 + (threadIdx.x >> 4);   // row
    if (i >= d || j >= d || (i >> 7) <= (j >> 7)) return;
    G[(size_t)i * d + j] = G[(size_t)j * d + i];
}

// VALU Gram: exact int64 replay for integer data (any |z - shift| < 2^31 with sums
// below 2^63), or fp64 for real-valued samples (shift = their mean, so the
// products are centred as in np.cov).  64 x 64 output tiles, 256 threads with 4 x 4
// outputs each, samples staged 16 at a time.
template <typename ZT, typename AT>
__global__ __launch_bounds__(256) void gram_val_kernel(const ZT* __restrict__ Z, int64_t ldz, int d,
                                                       int64_t n, int64_t kc, int nt,
                                                       const AT* __restrict__ shift, AT* __restrict__ G,
                                                       AT* __restrict__ S, const unsigned int* gate) {
    // gate (nullable): run only when the int8 packing flagged a value beyond two digits
    // (the exact replay of gram_planes, decided on the device)
    if (gate && !(*(const volatile unsigned int*)gate & kFlagI8Range)) return;
    constexpr int BT = 64, KS = 16;
    __shared__ AT As[KS][BT + 1], Bs[KS][BT + 1];
    const int tid = threadIdx.x;
    int ti, tj;
    tile_pair((int)blockIdx.x, nt, ti, tj);
    const bool diag = ti == tj;
    const int64_t k0 = (int64_t)blockIdx.y * kc;
    const int64_t k1 = k0 + kc < n ? k0 + kc : n;
    const int tr = (tid >> 4) * 4, tc = (tid & 15) * 4;
    AT acc[4][4] = {};
    AT zsum = 0;
    for (int64_t k = k0; k < k1; k += KS) {
        for (int e = tid; e < KS * BT; e += 256) {
            const int r = e / KS, kk = e % KS;
            const int gi = ti * BT + r, gj = tj * BT + r;
            const bool kok = k + kk < k1;
            As[kk][r] = (gi < d && kok) ? (AT)Z[(size_t)gi * ldz + k + kk] - (shift ? shift[gi] : (AT)0) : (AT)0;
            Bs[kk][r] = (gj < d && kok) ? (AT)Z[(size_t)gj * ldz + k + kk] - (shift ? shift[gj] : (AT)0) : (AT)0;
        }
        __syncthreads();
        if (diag && tid < BT)
            for (int kk = 0; kk < KS; ++kk) zsum += As[kk][tid];
#pragma unroll 4
        for (int kk = 0; kk < KS; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] += As[kk][tr + i] * Bs[kk][tc + j];
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int gi = ti * BT + tr + i, gj = tj * BT + tc + j;
            if (gi < d && gj < d && acc[i][j] != (AT)0) {
                atomic_add_val(G + (size_t)gi * d + gj, acc[i][j]);
                if (!diag) atomic_add_val(G + (size_t)gj * d + gi, acc[i][j]);
            }
        }
    if (diag && S && tid < BT && ti * BT + tid < d && zsum != (AT)0) atomic_add_val(S + ti * BT + tid, zsum);
}

// ------------------------------------------------------------ jump distances
// One wave per step t: lanes over the d coordinates of rows t and t+1.
template <typename XT>
__global__ __launch_bounds__(256) void jump_kernel(const XT* __restrict__ x, int64_t n, int d,
                                                   int64_t ld, double* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t + 1 >= n) return;
    const XT* r0 = x + (size_t)t * ld;
    const XT* r1 = r0 + ld;
    double acc = 0.0;
    for (int i = lane; i < d; i += 64) {
        const double df = as_f64(r1[i]) - as_f64(r0[i]);
        acc += df * df;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) out[t] = sqrt(acc);
}

// ------------------------------------------------------------ discrete marginal TVD
// Pass 1: per-coordinate min / max over both sets (integer-valued data; a
// non-integral fp64 value sets kFlagNonFinite).  Pass 2: per-coordinate counts in
// global memory (bins [min_i, max_i]).  Pass 3: one thread per coordinate sums
// |c1/n1 - c2/n2| over its bins in ascending value order -- the order of the
// reference's loop over np.unique (convergence_diag.py:35-46), so the result is
// bit-identical.
template <typename XT>
__device__ __forceinline__ bool to_i64(XT v, long long& o) {
    o = (long long)v;
    return true;
}
template <>
__device__ __forceinline__ bool to_i64<double>(double v, long long& o) {
    if (!(fabs(v) < 4.0e18) || v != rint(v)) return false;
    o = (long long)v;
    return true;
}

template <typename XT>
__global__ __launch_bounds__(256) void tvd_minmax_kernel(const XT* __restrict__ x, int64_t n, int d,
                                                         int64_t rows_per_block, long long* mn,
                                                         long long* mx, unsigned int* flags) {
    const int i = blockIdx.y * 256 + threadIdx.x;
    if (i >= d) return;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
    long long lo = 0x7fffffffffffffffLL, hi = -0x7fffffffffffffffLL - 1;
    bool bad = false;
    for (int64_t r = r0; r < r1; ++r) {
        long long v;
        if (!to_i64<XT>(x[(size_t)r * d + i], v)) {
            bad = true;
            continue;
        }
        lo = v < lo ? v : lo;
        hi = v > hi ? v : hi;
    }
    if (r1 > r0) {
        atomicMin(mn + i, lo);
        atomicMax(mx + i, hi);
    }
    if (bad) atomicOr(flags, kFlagNonFinite);
}

template <typename XT>
__global__ __launch_bounds__(256) void tvd_hist_kernel(const XT* __restrict__ x, int64_t n, int d,
                                                       int64_t rows_per_block, const long long* mn,
                                                       const long long* off, unsigned int* cnt) {
    const int i = blockIdx.y * 256 + threadIdx.x;
    if (i >= d) return;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
    const long long base = off[i] - mn[i];
    for (int64_t r = r0; r < r1; ++r) {
        long long v;
        if (to_i64<XT>(x[(size_t)r * d + i], v)) atomicAdd(cnt + base + v, 1u);
    }
}

__global__ __launch_bounds__(256) void tvd_sum_kernel(const unsigned int* __restrict__ c1,
                                                      const unsigned int* __restrict__ c2,
                                                      const long long* __restrict__ off, int d,
                                                      double n1, double n2, double* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= d) return;
    double acc = 0.0;
    for (long long b = off[i]; b < off[i + 1]; ++b) {
        const unsigned int a = c1[b], c = c2[b];
        if (a | c) acc += fabs((double)a / n1 - (double)c / n2);
    }
    out[i] = 0.5 * acc;
}

// ------------------------------------------------------------ binned histogram
// compute_tvd's histogram branch (convergence_diag.py:51-63): np.histogram with
// `bins` equal-width bins over a shared range.  Pass 1 (hist_range_*) finds each
// column's min / max in fp64 (integer data exact below 2^53) with 64-bit ordered
// keys; the host then builds the edges exactly as numpy does (np.linspace).
// Pass 2 bins every value with numpy's uniform-bin index arithmetic
// (numpy/lib/_histograms_impl.py: f = ((x - first) / denom) * bins, truncated,
// the last edge folded into the last bin, then the +-1 corrections against the
// linspace edges), so the counts are numpy's counts.  Small d x bins: counts in
// LDS per block (flattened element loop); otherwise one thread per column.
__device__ __forceinline__ long long f64_key(double v) {  // order-preserving int64 key
    const long long b = __double_as_longlong(v);
    return b ^ ((b >> 63) & 0x7fffffffffffffffLL);
}

template <typename XT>
__device__ __forceinline__ void range_one(XT v, long long& lo, long long& hi, bool& bad) {
    const double x = (double)v;
    if (!isfinite(x) || (sizeof(XT) == 8 && !std::is_same<XT, double>::value && fabs(x) > 9007199254740992.0)) {
        bad = true;
        return;
    }
    const long long k = f64_key(x);
    lo = k < lo ? k : lo;
    hi = k > hi ? k : hi;
}

template <typename XT>
__global__ __launch_bounds__(256) void hist_range_cols_kernel(const XT* __restrict__ x, int64_t n, int d,
                                                              int64_t rows_per_block, long long* mn,
                                                              long long* mx, unsigned int* flags) {
    const int i = blockIdx.y * 256 + threadIdx.x;
    if (i >= d) return;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
    long long lo = 0x7fffffffffffffffLL, hi = -0x7fffffffffffffffLL - 1;
    bool bad = false;
    for (int64_t r = r0; r < r1; ++r) range_one<XT>(x[(size_t)r * d + i], lo, hi, bad);
    if (r1 > r0) {
        atomicMin(mn + i, lo);
        atomicMax(mx + i, hi);
    }
    if (bad) atomicOr(flags, kFlagNonFinite);
}

// small d (<= kHistLdsCols): flattened grid-stride loop, per-block LDS keys
constexpr int kHistLdsCols = 512;
template <typename XT>
__global__ __launch_bounds__(256) void hist_range_flat_kernel(const XT* __restrict__ x, int64_t total, int d,
                                                              long long* mn, long long* mx,
                                                              unsigned int* flags) {
    __shared__ long long slo[kHistLdsCols], shi[kHistLdsCols];
    for (int i = threadIdx.x; i < d; i += 256) {
        slo[i] = 0x7fffffffffffffffLL;
        shi[i] = -0x7fffffffffffffffLL - 1;
    }
    __syncthreads();
    bool bad = false;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += stride) {
        long long lo = 0x7fffffffffffffffLL, hi = -0x7fffffffffffffffLL - 1;
        range_one<XT>(x[e], lo, hi, bad);
        if (lo <= hi) {
            const int i = (int)(e % d);
            atomicMin(slo + i, lo);
            atomicMax(shi + i, hi);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < d; i += 256) {
        if (slo[i] <= shi[i]) {
            atomicMin(mn + i, slo[i]);
            atomicMax(mx + i, shi[i]);
        }
    }
    if (bad) atomicOr(flags, kFlagNonFinite);
}

__global__ void hist_keys_to_f64_kernel(const long long* __restrict__ mn, const long long* __restrict__ mx,
                                        int d, double* __restrict__ lo, double* __restrict__ hi) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= d) return;
    auto un = [](long long k) { return __longlong_as_double(k ^ ((k >> 63) & 0x7fffffffffffffffLL)); };
    lo[i] = un(mn[i]);
    hi[i] = un(mx[i]);
}

// bin of one value (numpy's uniform-bin path; x already known to be in range)
__device__ __forceinline__ int64_t hist_bin(double x, const double* __restrict__ e, double first,
                                            double denom, int64_t nb) {
    const double f = ((x - first) / denom) * (double)nb;
    int64_t k = (int64_t)f;
    if (k == nb) k -= 1;
    if (x < e[k]) k -= 1;
    if (x >= e[k + 1] && k != nb - 1) k += 1;
    return k;
}

template <typename XT>
__global__ __launch_bounds__(256) void hist_cols_kernel(const XT* __restrict__ x, int64_t n, int d,
                                                        int64_t rows_per_block, int64_t nb,
                                                        const double* __restrict__ edges,
                                                        const double* __restrict__ fd,
                                                        unsigned long long* __restrict__ cnt) {
    const int i = blockIdx.y * 256 + threadIdx.x;
    if (i >= d) return;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
    const double* e = edges + (size_t)i * (nb + 1);
    const double first = fd[2 * i], denom = fd[2 * i + 1];
    const double lo = e[0], hi = e[nb];
    for (int64_t r = r0; r < r1; ++r) {
        const double v = (double)x[(size_t)r * d + i];
        if (v >= lo && v <= hi) atomicAdd(cnt + (size_t)i * nb + hist_bin(v, e, first, denom, nb), 1ull);
    }
}

constexpr int kHistLdsBins = 8192;
template <typename XT>
__global__ __launch_bounds__(256) void hist_flat_kernel(const XT* __restrict__ x, int64_t total, int d,
                                                        int64_t nb, const double* __restrict__ edges,
                                                        const double* __restrict__ fd,
                                                        unsigned long long* __restrict__ cnt) {
    __shared__ unsigned int sc[kHistLdsBins];
    const int nbins = d * (int)nb;
    for (int k = threadIdx.x; k < nbins; k += 256) sc[k] = 0u;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t e0 = (int64_t)blockIdx.x * 256 + threadIdx.x; e0 < total; e0 += stride) {
        const int i = (int)(e0 % d);
        const double* e = edges + (size_t)i * (nb + 1);
        const double v = (double)x[e0];
        if (v >= e[0] && v <= e[nb]) atomicAdd(sc + i * nb + hist_bin(v, e, fd[2 * i], fd[2 * i + 1], nb), 1u);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < nbins; k += 256)
        if (sc[k]) atomicAdd(cnt + k, (unsigned long long)sc[k]);
}

// ============================================================ launchers
namespace launch {

#define LGS_XT(xt, T, ...)       \
    do {                         \
        if ((xt) == 1) {         \
            using T = int32_t;   \
            __VA_ARGS__;         \
        } else if ((xt) == 2) {  \
            using T = int64_t;   \
            __VA_ARGS__;         \
        } else {                 \
            using T = double;    \
            __VA_ARGS__;         \
        }                        \
    } while (0)

hipError_t series_stats(const SeriesArgs& a, hipStream_t st) {
    if (a.n_series <= 0 || a.n <= 0) return hipSuccess;
    const int64_t gx = a.n_series < 65536 ? a.n_series : 65536;
    const dim3 grid((unsigned)gx, (unsigned)((a.n_series + gx - 1) / gx));
    LGS_XT(a.xtype, XT, hipLaunchKernelGGL(series_stats_kernel<XT>, grid, dim3(256), 0, st, a));
    return hipGetLastError();
}

int64_t gram_chunk(int64_t n, int nt) {
    const int64_t pairs = (int64_t)nt * (nt + 1) / 2;
    int64_t splits = (2048 + pairs - 1) / pairs;
    int64_t kc = (n + splits - 1) / splits;
    kc = (kc + 63) / 64 * 64;
    if (kc < 1024) kc = 1024;
    if (kc > 32768) kc = 32768;
    return kc;
}

hipError_t gram(const void* Z, int xtype, int64_t ldz, int d, int64_t n, const void* shift, void* G,
                void* S, hipStream_t st, const unsigned int* gate) {
    if (n <= 0 || d <= 0) return hipSuccess;
    const int nt = (d + 63) / 64;
    const int64_t kc = gram_chunk(n, nt);
    const dim3 grid((unsigned)(nt * (nt + 1) / 2), (unsigned)((n + kc - 1) / kc));
    if (xtype == 2)
        hipLaunchKernelGGL((gram_val_kernel<int64_t, long long>), grid, dim3(256), 0, st, (const int64_t*)Z, ldz, d, n, kc, nt, (const long long*)shift, (long long*)G, (long long*)S, gate);
    else if (xtype == 1)
        hipLaunchKernelGGL((gram_val_kernel<int32_t, long long>), grid, dim3(256), 0, st, (const int32_t*)Z, ldz, d, n, kc, nt, (const long long*)shift, (long long*)G, (long long*)S, gate);
    else
        hipLaunchKernelGGL((gram_val_kernel<double, double>), grid, dim3(256), 0, st, (const double*)Z, ldz, d, n, kc, nt, (const double*)shift, (double*)G, (double*)S, gate);
    return hipGetLastError();
}

hipError_t gram_pack(const void* X, int xtype, bool coord_major, int64_t ldx, int d, int64_t n,
                     const long long* shift, int8_t* Ph, int8_t* Pl, int64_t ldp, unsigned int* flags,
                     hipStream_t st) {
    const int dpad = (d + 127) / 128 * 128;
    const dim3 grid((unsigned)(ldp / 64), (unsigned)(dpad / 64));
    if (xtype == 2) {
        if (coord_major)
            hipLaunchKernelGGL((gram_pack_kernel<int64_t, true>), grid, dim3(256), 0, st, (const int64_t*)X, ldx, d, n, shift, Ph, Pl, ldp, flags);
        else
            hipLaunchKernelGGL((gram_pack_kernel<int64_t, false>), grid, dim3(256), 0, st, (const int64_t*)X, ldx, d, n, shift, Ph, Pl, ldp, flags);
    } else {
        if (coord_major)
            hipLaunchKernelGGL((gram_pack_kernel<int32_t, true>), grid, dim3(256), 0, st, (const int32_t*)X, ldx, d, n, shift, Ph, Pl, ldp, flags);
        else
            hipLaunchKernelGGL((gram_pack_kernel<int32_t, false>), grid, dim3(256), 0, st, (const int32_t*)X, ldx, d, n, shift, Ph, Pl, ldp, flags);
    }
    return hipGetLastError();
}

hipError_t gram_planes(const int8_t* Ph, const int8_t* Pl, int64_t ldp, int d, void* G, void* S,
                       hipStream_t st, const unsigned int* gate) {
    const int nt = (d + 127) / 128;
    const int64_t pairs = (int64_t)nt * (nt + 1) / 2;
    // about 2 workgroups (16 waves) per CU, K chunks of 64..16384 samples
    int64_t splits = (512 + pairs - 1) / pairs;
    int64_t kc = (ldp + splits - 1) / splits;
    kc = (kc + 63) / 64 * 64;
    if (kc > 16384) kc = 16384;
    if (kc < 64) kc = 64;
    const dim3 grid((unsigned)pairs, (unsigned)((ldp + kc - 1) / kc));
    hipLaunchKernelGGL(gram_planes_kernel, grid, dim3(512), 0, st, Ph, Pl, ldp, d, ldp, kc, nt,
                       (unsigned long long*)G, (unsigned long long*)S, gate);
    if (nt > 1)
        hipLaunchKernelGGL(gram_mirror_kernel, dim3((unsigned)((d + 15) / 16), (unsigned)((d + 15) / 16)),
                           dim3(256), 0, st, (unsigned long long*)G, d, gate);
    return hipGetLastError();
}

hipError_t jump(const void* x, int xtype, int64_t n, int d, int64_t ld, double* out, hipStream_t st) {
    if (n < 2) return hipSuccess;
    const dim3 grid((unsigned)((n - 1 + 3) / 4));
    LGS_XT(xtype, XT, hipLaunchKernelGGL(jump_kernel<XT>, grid, dim3(256), 0, st, (const XT*)x, n, d, ld, out));
    return hipGetLastError();
}

static int64_t tvd_rows(int64_t n) { return n < 256 ? 1 : (n + 1023) / 1024 < 64 ? 64 : (n + 1023) / 1024; }

hipError_t tvd_minmax(const void* x, int xtype, int64_t n, int d, long long* mn, long long* mx,
                      unsigned int* flags, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t rpb = tvd_rows(n);
    const dim3 grid((unsigned)((n + rpb - 1) / rpb), (unsigned)((d + 255) / 256));
    LGS_XT(xtype, XT, hipLaunchKernelGGL(tvd_minmax_kernel<XT>, grid, dim3(256), 0, st, (const XT*)x, n, d, rpb, mn, mx, flags));
    return hipGetLastError();
}

hipError_t tvd_hist(const void* x, int xtype, int64_t n, int d, const long long* mn,
                    const long long* off, unsigned int* cnt, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t rpb = tvd_rows(n);
    const dim3 grid((unsigned)((n + rpb - 1) / rpb), (unsigned)((d + 255) / 256));
    LGS_XT(xtype, XT, hipLaunchKernelGGL(tvd_hist_kernel<XT>, grid, dim3(256), 0, st, (const XT*)x, n, d, rpb, mn, off, cnt));
    return hipGetLastError();
}

hipError_t tvd_sum(const unsigned int* c1, const unsigned int* c2, const long long* off, int d,
                   int64_t n1, int64_t n2, double* out, hipStream_t st) {
    hipLaunchKernelGGL(tvd_sum_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, st, c1, c2, off, d,
                       (double)n1, (double)n2, out);
    return hipGetLastError();
}

static unsigned flat_blocks(int64_t total) {
    const int64_t b = (total + 4095) / 4096;  // ~16 elements per thread
    return (unsigned)(b < 1 ? 1 : b > 2048 ? 2048 : b);
}

hipError_t hist_range(const void* x, int xtype, int64_t n, int d, long long* mn, long long* mx,
                      unsigned int* flags, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (d <= kHistLdsCols) {
        const int64_t total = n * d;
        LGS_XT(xtype, XT, hipLaunchKernelGGL(hist_range_flat_kernel<XT>, dim3(flat_blocks(total)), dim3(256), 0, st, (const XT*)x, total, d, mn, mx, flags));
    } else {
        const int64_t rpb = tvd_rows(n);
        const dim3 grid((unsigned)((n + rpb - 1) / rpb), (unsigned)((d + 255) / 256));
        LGS_XT(xtype, XT, hipLaunchKernelGGL(hist_range_cols_kernel<XT>, grid, dim3(256), 0, st, (const XT*)x, n, d, rpb, mn, mx, flags));
    }
    return hipGetLastError();
}

hipError_t hist_keys_to_f64(const long long* mn, const long long* mx, int d, double* lo, double* hi,
                            hipStream_t st) {
    hipLaunchKernelGGL(hist_keys_to_f64_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, st, mn, mx, d, lo, hi);
    return hipGetLastError();
}

hipError_t hist_counts(const void* x, int xtype, int64_t n, int d, int64_t nb, const double* edges,
                       const double* fd, unsigned long long* cnt, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if ((int64_t)d * nb <= kHistLdsBins) {
        const int64_t total = n * d;
        LGS_XT(xtype, XT, hipLaunchKernelGGL(hist_flat_kernel<XT>, dim3(flat_blocks(total)), dim3(256), 0, st, (const XT*)x, total, d, nb, edges, fd, cnt));
    } else {
        const int64_t rpb = tvd_rows(n);
        const dim3 grid((unsigned)((n + rpb - 1) / rpb), (unsigned)((d + 255) / 256));
        LGS_XT(xtype, XT, hipLaunchKernelGGL(hist_cols_kernel<XT>, grid, dim3(256), 0, st, (const XT*)x, n, d, rpb, nb, edges, fd, cnt));
    }
    return hipGetLastError();
}

}  // namespace launch
}  // namespace lgs
