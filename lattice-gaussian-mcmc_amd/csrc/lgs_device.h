// lgs_device.h -- device-side building blocks of the Klein / IMHK path (gfx950).
//
//  * Philox4x32-10 counter RNG + NumPy's 53-bit double conversion: replaces the
//    single MT19937 draw of np.random.choice (reference src/samplers/klein.py:175)
//    and np.random.rand (src/samplers/imhk.py:167).  Counter layout: DESIGN.md §RNG.
//  * SampleZ: the 1-D discrete Gaussian of klein.py:101-179 (support window,
//    table, cumulative search) evaluated per lane.
//
// The translation unit is compiled with -ffp-contract=off: every a*b+c below is
// two roundings, exactly like NumPy, unless written as an explicit fma().
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lgs_kernels.h"

// Round-5 near-field trims of klein_mfma_kernel, on by default (LGS_R5_OFF: the
// round-4 forms, for A/B): the range checks and the sub-panel's nonzero flag from its
// extremes and Z stored through the row's uniform base (LGS_TAIL2), the SampleZ
// dispatch from the host's code in the record (LGS_DISP_CODE), the capped quantile
// test without short-circuit branches (LGS_CAP_BRANCHLESS), each coordinate's int16
// history value stored at once instead of packed through 8 registers
// (LGS_HIST_STORE16), and the tail's integer extremes / running history pointer
// (LGS_TAIL3).  Together 2.47 -> 2.32-2.37 ms per 2^18 C3 samples, identical outputs
// (profiles/r05f_kb_trims.log, r05h_kb.log).
#ifndef LGS_R5_OFF
#ifndef LGS_TAIL2
#define LGS_TAIL2 1
#endif
#ifndef LGS_DISP_CODE
#define LGS_DISP_CODE 1
#endif
#ifndef LGS_CAP_BRANCHLESS
#define LGS_CAP_BRANCHLESS 1
#endif
#ifndef LGS_HIST_STORE16
#define LGS_HIST_STORE16 1
#endif
#ifndef LGS_TAIL3  // (integer extremes, running history pointer, the uncovered mask behind a ballot)
#define LGS_TAIL3 1
#endif
#endif

namespace lgs {

// Basis constants are never written by a kernel: reading them through the
// constant address space lets wave-uniform loads be scalar (s_load).  Through a
// generic pointer the compiler cannot rule out aliasing with the coefficient
// stores and issues vector (or flat) loads with a full-latency wait each.
using cdptr = const __attribute__((address_space(4))) double*;
__device__ __forceinline__ cdptr cst(const double* p) { return (cdptr)p; }

constexpr uint32_t kTagCoord = 0;
constexpr uint32_t kTagAccept = 1;

struct U4 {
    uint32_t x, y, z, w;
};

template <bool OPAQUE = true>  // false: keys may live in VGPRs (divergent callers)
__device__ __forceinline__ U4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint32_t k0, uint32_t k1) {
#ifndef LGS_PHILOX_HOIST
    // opaque to loop-invariant motion: otherwise the 20 round keys of the (kernel-
    // constant) seed are hoisted out of the coordinate loop, spilled to VGPR lanes
    // and read back with v_readlane + s_nop at every call; recomputing them is 18 SALU
    // adds.  (readfirstlane: the keys are the same in every lane, and the compiler may
    // park them in a VGPR across a call)
    if constexpr (OPAQUE) {
        k0 = __builtin_amdgcn_readfirstlane(k0);
        k1 = __builtin_amdgcn_readfirstlane(k1);
        asm volatile("" : "+s"(k0), "+s"(k1));
        // likewise the first round's products of the per-lane (step, chain) words:
        // hoisted, they were spilled and reloaded from scratch at every draw
        asm volatile("" : "+v"(c1), "+v"(c2));
    }
#endif
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
#ifdef LGS_PHILOX_MAD64
        // one 32x32->64 multiply (v_mad_u64_u32) per product instead of mul_lo + mul_hi
        // (round 4: the mul_lo / mul_hi pair below takes 13 fewer spilled VGPRs in the
        // Klein kernel and runs it 2-4 % faster, profiles/r04ab_*, r04ac_*)
        const uint64_t m0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t m1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t lo0 = (uint32_t)m0, hi0 = (uint32_t)(m0 >> 32);
        const uint32_t lo1 = (uint32_t)m1, hi1 = (uint32_t)(m1 >> 32);
#else
        const uint32_t lo0 = 0xD2511F53u * c0;
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2);
#endif
#ifndef LGS_PHILOX_NO_BITOP3
        if (OPAQUE && r >= 2) {
            // from the third round every word is per-lane: each three-way xor in one gfx950
            // v_bitop3_b32 (truth table 0x96) instead of two v_xor_b32 -- 16 VALU fewer per
            // block, the same bits (the first two rounds mix scalar words: s_xor + v_xor)
            uint32_t n0, n2;
            asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n0) : "v"(hi1), "v"(c1), "s"(k0));
            asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n2) : "v"(hi0), "v"(c3), "s"(k1));
            c0 = n0;
            c1 = lo1;
            c2 = n2;
            c3 = lo0;
            continue;
        }
#endif
        const uint32_t n0 = hi1 ^ c1 ^ k0;
        const uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
    }
    return {c0, c1, c2, c3};
}

// NumPy legacy double: ((a >> 5) * 2^26 + (b >> 6)) / 2^53 (exact in fp64).
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// Uniform of the IMHK acceptance test (ctr = {0, step, chain, 1}).
__device__ __forceinline__ double accept_uniform(uint64_t seed, uint32_t step, uint32_t chain) {
    U4 w = philox4x32_10(0u, step, chain, kTagAccept, (uint32_t)seed, (uint32_t)(seed >> 32));
    return u53(w.x, w.y);
}

// Per-lane coordinate uniform stream: slot k = d-1-i, two slots per Philox call.
template <bool OPAQUE = true>
struct CoordStreamT {
    uint32_t k0, k1, step, chain;
    uint32_t pair;  // cached pair index (0xffffffff = none); LGS_PHILOX2 (OPAQUE): cached quad index
    U4 w;
#ifdef LGS_PHILOX2
    U4 w2;  // the quad's second pair
#endif
#ifdef LGS_PHILOX_NEXT
    U4 wn;          // the next pair's block, drawn at the current pair's second slot
    uint32_t pn;    // its pair index (0xffffffff = none)
#endif
    __device__ __forceinline__ void init(uint64_t seed, uint32_t step_, uint32_t chain_) {
        k0 = (uint32_t)seed;
        k1 = (uint32_t)(seed >> 32);
        step = step_;
        chain = chain_;
        pair = 0xffffffffu;
#ifdef LGS_PHILOX_NEXT
        pn = 0xffffffffu;
#endif
    }
    __device__ __forceinline__ double u(uint32_t slot) {
#ifdef LGS_DIAG_CHEAP_RNG  // diagnostic builds only: Philox cost probe (wrong stream)
        uint32_t hh = (slot * 0x9E3779B9u) ^ (chain * 0x85EBCA6Bu) ^ step ^ k0;
        hh ^= hh >> 15;
        hh *= 0x2C1B3C6Du;
        hh ^= hh >> 12;
        return (double)hh * 0x1p-32;
#endif
#ifdef LGS_PHILOX2
        // the Klein kernels' wave-uniform slots: the two Philox blocks of a quad of
        // slots (4 coordinates) computed together -- two independent 10-round chains
        // the scheduler interleaves -- behind a scalar test (the cache key is uniform)
        if constexpr (OPAQUE) {
            const uint32_t q = __builtin_amdgcn_readfirstlane(slot >> 2);
            if (q != __builtin_amdgcn_readfirstlane(pair)) {
                w = philox4x32_10<true>(2 * q, step, chain, kTagCoord, k0, k1);
                w2 = philox4x32_10<true>(2 * q + 1, step, chain, kTagCoord, k0, k1);
                pair = q;
            }
            const U4 ww = (slot & 2u) ? w2 : w;
            return (slot & 1u) ? u53(ww.z, ww.w) : u53(ww.x, ww.y);
        }
#endif
#ifdef LGS_PHILOX_NEXT
        // software-pipelined (the Klein kernels' wave-uniform slots, ascending): the block
        // of pair p + 1 is drawn at pair p's second slot, a step before its first use,
        // off that step's decision chain; a slot sequence that jumps (skipped
        // sub-panels) draws its block in place
        if constexpr (OPAQUE) {
            const uint32_t p = __builtin_amdgcn_readfirstlane(slot >> 1);
            if (p != __builtin_amdgcn_readfirstlane(pair)) {
                if (p == __builtin_amdgcn_readfirstlane(pn))
                    w = wn;
                else
                    w = philox4x32_10<true>(p, step, chain, kTagCoord, k0, k1);
                pair = p;
            }
            const double r = (slot & 1u) ? u53(w.z, w.w) : u53(w.x, w.y);
            if (slot & 1u) {
                wn = philox4x32_10<true>(p + 1, step, chain, kTagCoord, k0, k1);
                pn = p + 1;
            }
            return r;
        }
#endif
        const uint32_t p = slot >> 1;
        if (p != pair) {
            w = philox4x32_10<OPAQUE>(p, step, chain, kTagCoord, k0, k1);
            pair = p;
        }
        return (slot & 1u) ? u53(w.z, w.w) : u53(w.x, w.y);
    }
};
using CoordStream = CoordStreamT<true>;

// ------------------------------------------------------------------ SampleZ
// Support window of _compute_1d_probabilities (klein.py:113-128).
__device__ __forceinline__ void support_window(double mu, double sig, int precision, int64_t& lo,
                                               int64_t& hi) {
    const double rf = (sig < 0.1) ? (double)(precision > 3 ? precision : 3) : (double)precision;
    lo = (int64_t)floor(mu - rf * sig);
    hi = (int64_t)ceil(mu + rf * sig);
    if (hi - lo > 1000) {
        const int64_t c = (int64_t)rint(mu);  // np.round: half to even
        lo = c - 500;
        hi = c + 500;
    }
}

struct SampleZOut {
    int64_t z;
    double log_norm;  // log sum_k exp(-(k-mu)^2/(2 sig^2)) over the window (Wang-Ling weight)
};

// ---------------------------------------------------------- certified decisions
// The blocked Klein kernels form mu_i in another fp64 order than the reference
// (blocked FMA / MFMA sums, the int8-digit far field, a reciprocal of R_ii instead
// of the division of klein.py:191-195).  Every SampleZ function below takes dmu:
//   dmu < 0   decide at mu (the reference-order kernel, or a redo);
//   dmu >= 0  a rigorous bound on |mu - mu_ref| (lgs_set_basis: kSzCa / kSzCb):
//             the decision is returned only when it is the same for EVERY mean
//             within dmu of mu -- the support window stays put and u stays clear
//             of every CDF boundary the shift can move -- else kAmbZ / kAmbiguous,
//             and the kernel recomputes mu in the reference's order for that
//             coordinate (mu_exact_col) and decides again with dmu < 0.
// Boundary motion: a mean shift of dmu changes log w_k = -(k-mu)^2/(2 s^2) by
// (k - mu) dmu / s^2 - dmu^2 / (2 s^2); the k-independent part cancels in every
// ratio, so the odds C_b / (S - C_b) of a CDF boundary move by a factor of at most
// E = e^dg, dg = (hi - lo) dmu / s^2 over a window [lo, hi].  Wide windows (s >= 4)
// use |dP/dmu| = |Cov(k, 1{k<=b})| / s^2 <= sd(k) / (2 s^2) <= 0.6 / s instead.  A
// 1e-13 S (1e-12 S on the Euler-Maclaurin path) margin covers the rounding of the
// two evaluations.
constexpr int64_t kAmbZ = INT64_MIN;
constexpr double kAmbiguous = __builtin_inf();

// floor(mu - w) and ceil(mu + w) are the same for every mean within dmu of mu
__device__ __forceinline__ bool ends_stable(double mu, double w, double dmu) {
    const double tol = 1.01 * dmu + 4.5e-16 * (fabs(mu) + w + 1.0);
    const double x0 = mu - w, x1 = mu + w;
    return fabs(x0 - rint(x0)) > tol && fabs(x1 - rint(x1)) > tol;
}
// rint(mu) is the same for every mean within dmu of mu (m = mu - rint(mu) is exact)
__device__ __forceinline__ bool round_stable(double mu, double dmu) {
    return fabs(mu - rint(mu)) + 1.01 * dmu < 0.5;
}
// u S stays on its side of the CDF value Cb (0 <= Cb <= S) when the boundary's odds
// Cb / (S - Cb) move by a factor of at most E: target (S - Cb) vs E (S - target) Cb
// (their difference at E = 1 is S (target - Cb))
__device__ __forceinline__ bool boundary_clear(double target, double Cb, double S, double E) {
    const double a = target * (S - Cb), b = (S - target) * Cb;
    return (target > Cb ? a - E * b : b - E * a) > 1e-13 * (S * S);
}
// E >= e^dg (fp32 exp2 with the argument and result padded for its rounding);
// dg beyond the fp32 range gives +inf (nothing is clear)
__device__ __forceinline__ double odds_factor(double dg) {
    const float x = (float)(fma(dg, 1.4426950408889634 * 1.000001, 1e-6));
    return (double)exp2f(x) * 1.000001;
}
// support_window (below) is the same for every mean within dmu of mu
__device__ __forceinline__ bool window_stable(double mu, double sig, int precision, double dmu) {
    const double rf = (sig < 0.1) ? (double)(precision > 3 ? precision : 3) : (double)precision;
    if (!ends_stable(mu, rf * sig, dmu)) return false;
    const double lo = floor(mu - rf * sig), hi = ceil(mu + rf * sig);
    return !(hi - lo > 1000.0) || round_stable(mu, dmu);
}

// Decision of klein.py:143-179 for uniform u: the smallest k in the window with
// cumsum(p)[k] > u * sum(p), p_k proportional to exp(-((k-mu)/sig)^2 / 2).
// The table is max-shifted (w = 1 at the k nearest mu) instead of normalised by
// scipy's logsumexp: the normalisation cancels in cdf = cumsum / cumsum[-1], so
// the decision is the reference's up to ulp-level rounding of the boundaries.
// Two passes over the window (sum, then cumulative walk); no table storage.
__device__ __noinline__ SampleZOut sample_z_table(double mu, double sig, int precision,
                                                  bool linear_probs, double u,
                                                  bool want_log = true, double dmu = -1.0) {
    int64_t lo, hi;
    support_window(mu, sig, precision, lo, hi);
    int64_t ks = (int64_t)rint(mu);
    ks = ks < lo ? lo : (ks > hi ? hi : ks);
    const double ts = ((double)ks - mu) / sig;
    const double shift = -0.5 * (ts * ts);
    SampleZOut out;
    const double E = dmu >= 0.0 ? odds_factor((double)(hi - lo) * dmu / (sig * sig)) : 1.0;
    if (dmu >= 0.0 && (!window_stable(mu, sig, precision, dmu) || (linear_probs && shift < -700.0))) {
        out.z = kAmbZ;
        out.log_norm = 0.0;
        return out;
    }
    if (linear_probs && exp(shift) == 0.0) {
        // use_log_space=False: every probability underflows -> NaN -> the
        // reference's ValueError fallback round(mean) (klein.py:176-179).
        out.z = (int64_t)rint(mu);
        out.log_norm = -INFINITY;
        return out;
    }
    const double flo = (double)lo;
    const int n = (int)(hi - lo) + 1;
    double S = 0.0;
    for (int k = 0; k < n; ++k) {
        const double t = ((flo + (double)k) - mu) / sig;
        S += exp(-0.5 * (t * t) - shift);
    }
    const double target = u * S;
    double C = 0.0, Cp = 0.0;
    int64_t z = hi;
    for (int k = 0; k < n; ++k) {
        const double t = ((flo + (double)k) - mu) / sig;
        Cp = C;
        C += exp(-0.5 * (t * t) - shift);
        if (C > target) {
            z = lo + k;
            break;
        }
    }
    if (dmu >= 0.0 && ((z > lo && !boundary_clear(target, Cp, S, E)) ||
                       (z < hi && !boundary_clear(target, C, S, E)))) {
        out.z = kAmbZ;
        out.log_norm = 0.0;
        return out;
    }
    out.z = z;
    out.log_norm = want_log ? shift + log(S) : 0.0;
    return out;
}

// ------------------------------------------------------------ SampleZ, O(1)
// For sigma >= kEMMin the window sums are evaluated in closed form with the
// Euler-Maclaurin formula instead of a table walk:
//   sum_{j=a}^{b} f(j) = P(b) - P(a) + (f(a) + f(b)) / 2,
//   P(x) = sigma*sqrt(pi/2)*erf(t/sqrt2) - f(x) * sum_{m=1..6} c_m He_{2m-1}(t) / sigma^(2m-1),
//   f(x) = exp(-t^2/2), t = (x - mu)/sigma, c_m = B_2m/(2m)!.
// The remainder is < 1e-19 S for sigma >= 4 (|B_2m|/(2m)! ~ 2/(2pi)^2m), and
// the fp64 evaluation error was measured at < 1e-15 S over sigma in [4, 1e6]
// (DESIGN.md §SampleZ), the same order as the reference's own cumsum rounding.
// The decision k is located from erfinv of the target and corrected by +-1
// steps using C(k) - C(k-1) = f(k).  A draw whose margin to a CDF boundary is
// below 1e-12 S is recomputed by the table walk.
constexpr double kEMMin = 4.0;
constexpr double kSqrtHalfPi = 1.2533141373155003;  // sqrt(pi/2)
constexpr double kInvSqrt2 = 0.7071067811865476;
constexpr double kSqrt2 = 1.4142135623730951;

__device__ __forceinline__ double em_H(double t, double is) {
    const double c[6] = {1.0 / 12.0, -1.0 / 720.0, 1.0 / 30240.0, -1.0 / 1209600.0,
                         1.0 / 47900160.0, -5.284190138687493e-10};
    const double is2 = is * is;
    double hm = 1.0, h = t;  // He_0, He_1
    double p = is, res = 0.0;
    double n = 1.0;
#pragma unroll
    for (int m = 0; m < 6; ++m) {
        res = fma(c[m] * p, h, res);
        double h2 = fma(t, h, -n * hm);  // He_{n+1}
        n += 1.0;
        hm = h;
        h = h2;
        h2 = fma(t, h, -n * hm);  // He_{n+2}
        n += 1.0;
        hm = h;
        h = h2;
        p *= is2;
    }
    return res;
}

__device__ __noinline__ double em_P(double x, double mu, double sig, double is, double& fx) {
    const double t = (x - mu) * is;
    fx = exp(-0.5 * (t * t));
    return fma(-em_H(t, is), fx, sig * kSqrtHalfPi * erf(t * kInvSqrt2));
}

// Branch-free erf / Gaussian for the Euler-Maclaurin path.  etab holds, for
// y_j = j/64 (j = 0..kErfTabLast = 512), the correctly rounded pair {erf(y_j),
// exp(-y_j^2)} (filled on the host in long double, lgs_create).  With
// h = y - y_j, |h| <= 1/128:
//   erf(y)    = erf(y_j) + 2/sqrt(pi) e^{-y_j^2} sum_{n=1..7} (-1)^{n-1} H_{n-1}(y_j) h^n/n!
//   e^{-y^2}  = e^{-y_j^2} exp(-(2 y_j h + h^2)),  |2 y_j h + h^2| <= 0.26,
// (H_n physicists' Hermite polynomials; truncation < 1e-19 and < 1e-17 relative),
// so both cost a 16-byte table load and ~30 FMAs, with no data-dependent
// branches (ocml's erf selects one of several polynomials per lane).
// |y| > 8 returns (sign 1, 0): erfc(8) = 1e-29 and e^{-64} = 2e-28 are far below
// the fp64 resolution of S >= 10 (sigma >= 4).  The table (8.2 KB) is read from
// LDS in the Klein kernels (TP = lds pointer) and from global memory elsewhere.
using lds_cdptr = const __attribute__((address_space(3))) double*;
// Global-address-space pointer: global_load (vmcnt only) instead of flat_load,
// which also counts against lgkmcnt.
using gdptr = const __attribute__((address_space(1))) double*;

struct ErfExp {
    double erf, g;  // erf(y), exp(-y^2)
};

template <typename TP>
__device__ __forceinline__ ErfExp erf_gauss(double y, TP etab) {
    const double ay = fmin(fabs(y), 8.0);
    const double jd = rint(ay * 64.0);
    const int j = (int)jd;
    const double y0 = jd * (1.0 / 64.0);
    const double h = ay - y0;
    const double F = etab[2 * j], G = etab[2 * j + 1];
    const double y2 = y0 + y0;
    const double H1 = y2;
    const double H2 = fma(y2, H1, -2.0);
    const double H3 = fma(y2, H2, -4.0 * H1);
    const double H4 = fma(y2, H3, -6.0 * H2);
    const double H5 = fma(y2, H4, -8.0 * H3);
    const double H6 = fma(y2, H5, -10.0 * H4);
    double q = fma(-h * (1.0 / 7.0), H6, H5);
    q = fma(-h * (1.0 / 6.0), q, H4);
    q = fma(-h * (1.0 / 5.0), q, H3);
    q = fma(-h * (1.0 / 4.0), q, H2);
    q = fma(-h * (1.0 / 3.0), q, H1);
    q = fma(-h * 0.5, q, 1.0);
    const double e = fma(1.1283791670955126 * G, h * q, F);  // 2/sqrt(pi)
    // exp(-x), x = 2 y0 h + h^2 in [-0.26, 0.26]: degree-12 Taylor
    const double x = -fma(y2, h, h * h);
    double p = fma(x, 1.0 / 479001600.0, 1.0 / 39916800.0);
    p = fma(x, p, 1.0 / 3628800.0);
    p = fma(x, p, 1.0 / 362880.0);
    p = fma(x, p, 1.0 / 40320.0);
    p = fma(x, p, 1.0 / 5040.0);
    p = fma(x, p, 1.0 / 720.0);
    p = fma(x, p, 1.0 / 120.0);
    p = fma(x, p, 1.0 / 24.0);
    p = fma(x, p, 1.0 / 6.0);
    p = fma(x, p, 0.5);
    p = fma(x, p, 1.0);
    p = fma(x, p, 1.0);
    const bool big = fabs(y) > 8.0;
    ErfExp r;
    r.erf = copysign(big ? 1.0 : e, y);
    r.g = big ? 0.0 : G * p;
    return r;
}

// Coefficient form of the same table (used by the 32-row-panel Klein kernel):
// per grid point y0 = j/64, 18 doubles: the Taylor coefficients in h = y - y0 of
// erf (a0 = erf(y0), a_n = 2/sqrt(pi) (-1)^(n-1) H_{n-1}(y0) e^{-y0^2}/n!, n <= 7)
// and of e^{-y^2} (b_n = (-1)^n H_n(y0) e^{-y0^2}/n!, n <= 8), from long double on
// the host.  Two Horner chains on loaded coefficients: no fp64 constants to
// materialise (each costs two scalar moves per use), half the VALU work.
struct CoefTab {
    const double* __restrict__ p;
};

__device__ __forceinline__ ErfExp erf_gauss(double y, CoefTab tab) {
    typedef double d2v __attribute__((ext_vector_type(2)));
    const double ay = fmin(fabs(y), 8.0);
    const double jd = rint(ay * 64.0);
    const int j = (int)jd;
    const double h = ay - jd * (1.0 / 64.0);
    const d2v* c = (const d2v*)(tab.p + (size_t)j * kCoefStride);
    const d2v v0 = c[0], v1 = c[1], v2 = c[2], v3 = c[3];
    const d2v v4 = c[4], v5 = c[5], v6 = c[6], v7 = c[7], v8 = c[8];
    double e = fma(v3[1], h, v3[0]);
    e = fma(e, h, v2[1]);
    e = fma(e, h, v2[0]);
    e = fma(e, h, v1[1]);
    e = fma(e, h, v1[0]);
    e = fma(e, h, v0[1]);
    e = fma(e, h, v0[0]);
    double g = fma(v8[0], h, v7[1]);
    g = fma(g, h, v7[0]);
    g = fma(g, h, v6[1]);
    g = fma(g, h, v6[0]);
    g = fma(g, h, v5[1]);
    g = fma(g, h, v5[0]);
    g = fma(g, h, v4[1]);
    g = fma(g, h, v4[0]);
    const bool big = fabs(y) > 8.0;
    ErfExp r;
    r.erf = copysign(big ? 1.0 : e, y);
    r.g = big ? 0.0 : g;
    return r;
}

// Series form for |y| <= 1 (capped windows with sigma >= 360: |k - mu| <= 500.5
// gives |y| <= 0.983): erf(y) = 2/sqrt(pi) sum_{n<=17} (-1)^n y^(2n+1)/(n! (2n+1))
// and e^{-y^2} = sum_{n<=18} (-y^2)^n/n!, truncation < 5e-18 and < 1e-17, within
// 3e-16 / 5e-16 relative of libm over [0, 1] -- no table lookup (a gather whose
// latency sits on the decision's dependency chain), two independent Horner chains.
struct PolyErf {};
__device__ __forceinline__ ErfExp erf_gauss(double y, PolyErf) {
    const double z = y * y;
    double e = -9.063970842808673e-17;
    e = fma(e, z, 1.6342614095367152e-15);
    e = fma(e, z, -2.7835162072109215e-14);
    e = fma(e, z, 4.4632242632864775e-13);
    e = fma(e, z, -6.7113668551641105e-12);
    e = fma(e, z, 9.422759064650411e-11);
    e = fma(e, z, -1.2290555301717928e-09);
    e = fma(e, z, 1.4807192815879218e-08);
    e = fma(e, z, -1.6365844691234924e-07);
    e = fma(e, z, 1.6462114365889248e-06);
    e = fma(e, z, -1.492565035840625e-05);
    e = fma(e, z, 0.00012055332981789664);
    e = fma(e, z, -0.0008548327023450853);
    e = fma(e, z, 0.005223977625442188);
    e = fma(e, z, -0.026866170645131252);
    e = fma(e, z, 0.11283791670955126);
    e = fma(e, z, -0.37612638903183754);
    e = fma(e, z, 1.1283791670955126);
    double g = 1.5619206968586225e-16;
    g = fma(g, z, -2.8114572543455206e-15);
    g = fma(g, z, 4.779477332387385e-14);
    g = fma(g, z, -7.647163731819816e-13);
    g = fma(g, z, 1.1470745597729725e-11);
    g = fma(g, z, -1.6059043836821613e-10);
    g = fma(g, z, 2.08767569878681e-09);
    g = fma(g, z, -2.505210838544172e-08);
    g = fma(g, z, 2.755731922398589e-07);
    g = fma(g, z, -2.7557319223985893e-06);
    g = fma(g, z, 2.48015873015873e-05);
    g = fma(g, z, -0.0001984126984126984);
    g = fma(g, z, 0.001388888888888889);
    g = fma(g, z, -0.008333333333333333);
    g = fma(g, z, 0.041666666666666664);
    g = fma(g, z, -0.16666666666666666);
    g = fma(g, z, 0.5);
    g = fma(g, z, -1.0);
    g = fma(g, z, 1.0);
    ErfExp r;
    r.erf = y * e;
    r.g = g;
    return r;
}

// P(x) of the Euler-Maclaurin formula with NT Hermite correction terms
// (NT = 6 for sigma < 50; 3 suffice above: the next term is < 1e-18 S).
#define LGS_EM_ATTR __device__ __forceinline__
template <int NT, typename TP>
LGS_EM_ATTR double em_P_tab(double x, double mu, double sig, double is, TP etab, double& fx) {
    const double t = (x - mu) * is;
    const ErfExp ee = erf_gauss(t * kInvSqrt2, etab);
    fx = ee.g;
    const double c[6] = {1.0 / 12.0, -1.0 / 720.0, 1.0 / 30240.0, -1.0 / 1209600.0,
                         1.0 / 47900160.0, -5.284190138687493e-10};
    const double is2 = is * is;
    double hm = 1.0, h = t, p = is, res = 0.0, n = 1.0;
#pragma unroll
    for (int m = 0; m < NT; ++m) {
        res = fma(c[m] * p, h, res);
        if (m + 1 < NT) {
            double h2 = fma(t, h, -n * hm);
            n += 1.0;
            hm = h;
            h = h2;
            h2 = fma(t, h, -n * hm);
            n += 1.0;
            hm = h;
            h = h2;
            p *= is2;
        }
    }
    return fma(-res, fx, sig * kSqrtHalfPi * ee.erf);
}

template <typename TP>
LGS_EM_ATTR double gauss_tab(double kd, double mu, double is, TP etab) {
    return erf_gauss((kd - mu) * is * kInvSqrt2, etab).g;
}

// Euler-Maclaurin decision with the tabulated erf/exp.  The initial guess uses
// fp32 erfinvf (its error is absorbed by the +-1 steps); the decision rule,
// margins and table fallback are those of the libm path below.
template <int NT, typename TP>
__device__ __forceinline__ SampleZOut sample_z_em_tab(double mu, double sig, int precision,
                                                      bool linear_probs, double u, bool want_log,
                                                      int64_t lo, int64_t hi, TP etab, double dmu) {
    const double is = 1.0 / sig;
    double fL, fU, fk;
    const double PL = em_P_tab<NT>((double)lo, mu, sig, is, etab, fL);
    const double PU = em_P_tab<NT>((double)hi, mu, sig, is, etab, fU);
    const double S = (PU - PL) + 0.5 * (fL + fU);
    const double target = u * S;
    const double base = PL - 0.5 * fL;
    const float arg = fminf(fmaxf((float)((target + base) / (sig * kSqrtHalfPi)), -1.0f + 0x1p-24f),
                            1.0f - 0x1p-24f);
    const double x = mu + sig * kSqrt2 * (double)erfinvf(arg);
    double kd = fmin(fmax(ceil(x - 0.5), (double)lo), (double)hi);
    double Ck = em_P_tab<NT>(kd, mu, sig, is, etab, fk) + 0.5 * fk - base;
    const double fhi = (double)hi, flo = (double)lo;
    for (int it = 0; it < 64 && Ck <= target && kd < fhi; ++it) {  // move up
        kd += 1.0;
        fk = gauss_tab(kd, mu, is, etab);
        Ck += fk;
    }
    for (int it = 0; it < 64 && kd > flo && Ck - fk > target; ++it) {  // move down
        Ck -= fk;
        kd -= 1.0;
        fk = gauss_tab(kd, mu, is, etab);
    }
    const double margin = fmin(Ck - target, kd > flo ? target - (Ck - fk) : target);
    SampleZOut out;
    if (dmu >= 0.0) {  // certified: every mean within dmu decides the same
        if (!(margin > fma(0.6 * dmu, is, 1e-12) * S) || !(Ck > target) ||
            !window_stable(mu, sig, precision, dmu)) {
            out.z = kAmbZ;
            out.log_norm = 0.0;
            return out;
        }
    } else if (!(margin > 1e-12 * S) || !(Ck > target)) {
        return sample_z_table(mu, sig, precision, linear_probs, u, want_log);
    }
    out.z = (int64_t)kd;
    out.log_norm = want_log ? log(S) : 0.0;
    return out;
}

// Not inlined: inlining lets the compiler hoist the ~100 polynomial constants of
// erf/erfinv/exp/log out of the coordinate loop into registers (measured: 398
// VGPR+AGPR, 1 wave/SIMD); as a call the kernel stays at <= 170 VGPRs.
#ifndef LGS_SAMPLEZ_INLINE
#define LGS_SAMPLEZ_ATTR __device__ __noinline__
#else
#define LGS_SAMPLEZ_ATTR __device__ __forceinline__
#endif
// Windows of at most 4 points (sigma < 0.1 gives at most 3): exponents first,
// max-shift, and exp() only for the terms that do not underflow relative to the
// largest (e - e_max < -745.2 gives exactly 0.0 in fp64, as exp would), so the
// common near-deterministic case costs one exponent per point and no exp.
// Same decision rule as sample_z_table: smallest k with cumsum > u * sum.
__device__ __forceinline__ bool sample_z_small(double mu, double sig, int precision,
                                               bool linear_probs, double u, bool want_log,
                                               SampleZOut& out, double dmu) {
    int64_t lo, hi;
    support_window(mu, sig, precision, lo, hi);
    if (hi - lo > 3) return false;
    const int n = (int)(hi - lo) + 1;
    const double is = 1.0 / sig;
    double e[4];
    double emax = -INFINITY;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double t = (((double)lo + (double)k) - mu) * is;
        e[k] = k < n ? -0.5 * (t * t) : -INFINITY;
        emax = fmax(emax, e[k]);
    }
    if (dmu >= 0.0 && (!window_stable(mu, sig, precision, dmu) || (linear_probs && emax < -700.0))) {
        out.z = kAmbZ;
        out.log_norm = 0.0;
        return true;
    }
    if (linear_probs && emax < -745.2) {  // every probability underflows: round(mean)
        out.z = (int64_t)rint(mu);
        out.log_norm = -INFINITY;
        return true;
    }
    double w[4];
    double S = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double x = e[k] - emax;
        w[k] = x == 0.0 ? 1.0 : (x < -745.2 ? 0.0 : exp(x));
        S += w[k];
    }
    const double target = u * S;
    double C = 0.0, Cp = 0.0, Cz = S;
    int64_t z = hi;
    bool found = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double Cn = C + w[k];
        if (!found && k < n && Cn > target) {
            z = lo + k;
            found = true;
            Cp = C;
            Cz = Cn;
        }
        C = Cn;
    }
    if (dmu >= 0.0) {
        const double E = odds_factor((double)(hi - lo) * dmu * (is * is));
        if ((z > lo && !boundary_clear(target, Cp, S, E)) || (z < hi && !boundary_clear(target, Cz, S, E))) {
            out.z = kAmbZ;
            out.log_norm = 0.0;
            return true;
        }
    }
    out.z = z;
    out.log_norm = want_log ? emax + log(S) : 0.0;
    return true;
}

// etab == nullptr selects the libm Euler-Maclaurin path (ocml erf/exp/erfinv).
LGS_SAMPLEZ_ATTR SampleZOut sample_z(double mu, double sig, int precision, bool linear_probs,
                                     double u, bool want_log, const double* __restrict__ etab,
                                     double dmu = -1.0) {
    if (sig < kEMMin) {
        SampleZOut o;
        if (sample_z_small(mu, sig, precision, linear_probs, u, want_log, o, dmu)) return o;
        return sample_z_table(mu, sig, precision, linear_probs, u, want_log, dmu);
    }
    int64_t lo, hi;
    support_window(mu, sig, precision, lo, hi);
    if (etab) {
        return sig < 50.0 ? sample_z_em_tab<6>(mu, sig, precision, linear_probs, u, want_log, lo, hi, etab, dmu)
                          : sample_z_em_tab<3>(mu, sig, precision, linear_probs, u, want_log, lo, hi, etab, dmu);
    }
    const double is = 1.0 / sig;
    double fL, fU, fk;
    const double PL = em_P((double)lo, mu, sig, is, fL);
    const double PU = em_P((double)hi, mu, sig, is, fU);
    const double S = (PU - PL) + 0.5 * (fL + fU);
    const double target = u * S;
    const double base = PL - 0.5 * fL;  // C(k) = P(k) + f(k)/2 - base
    double arg = (target + base) / (sig * kSqrtHalfPi);
    arg = fmin(fmax(arg, -1.0 + 0x1p-53), 1.0 - 0x1p-53);
    const double x = mu + sig * kSqrt2 * erfinv(arg);
    double kd = ceil(x - 0.5);
    kd = fmin(fmax(kd, (double)lo), (double)hi);
    double Ck = em_P(kd, mu, sig, is, fk) + 0.5 * fk - base;
    const double fhi = (double)hi, flo = (double)lo;
    for (int it = 0; it < 64 && Ck <= target && kd < fhi; ++it) {  // move up
        kd += 1.0;
        const double t = (kd - mu) * is;
        fk = exp(-0.5 * (t * t));
        Ck += fk;
    }
    for (int it = 0; it < 64 && kd > flo && Ck - fk > target; ++it) {  // move down
        Ck -= fk;
        kd -= 1.0;
        const double t = (kd - mu) * is;
        fk = exp(-0.5 * (t * t));
    }
    const double margin = fmin(Ck - target, kd > flo ? target - (Ck - fk) : target);
    SampleZOut out;
    if (dmu >= 0.0) {
        if (!(margin > fma(0.6 * dmu, is, 1e-12) * S) || !(Ck > target) ||
            !window_stable(mu, sig, precision, dmu)) {
            out.z = kAmbZ;
            out.log_norm = 0.0;
            return out;
        }
    } else if (!(margin > 1e-12 * S) || !(Ck > target)) {
        return sample_z_table(mu, sig, precision, linear_probs, u, want_log);
    }
    out.z = (int64_t)kd;
    out.log_norm = want_log ? log(S) : 0.0;
    return out;
}

// ------------------------------------------------- SampleZ on the Klein path
// Same decisions as sample_z, using the per-coordinate constants q (layout:
// lgs_kernels.h kSzc*): no divisions, no 64-bit integer arithmetic, and for
// the wide windows the two window-end evaluations of S and base are replaced by
// the closed form (uncapped, rf >= 9: the tails beyond +-9 sigma are < 1e-18 S)
// or by host-fitted polynomials in m = mu - rint(mu) (capped windows; fitted
// and checked to 4e-17 S in long double, lgs_capi.hip build_szc).  Returns z as
// an exact fp64 integer.
template <int NT, typename TP>
__device__ __forceinline__ double em_C_rel(double kd, double m, double sig, double is, TP etab,
                                           double base, double& fk) {
    // C(k) = P(k) + f(k)/2 - base with k - mu = kd - m (exact to one rounding)
    return em_P_tab<NT>(kd, m, sig, is, etab, fk) + 0.5 * fk - base;
}

// q[0..8] of a coordinate, loaded as one batch before any branch on them: one
// memory round trip instead of one per branch level (the kind, then the window, ...)
struct QHead {
    double v[9];
};
template <typename QP>
__device__ __forceinline__ QHead load_head(QP q) {
    QHead h;
#pragma unroll
    for (int k = 0; k < 9; ++k) h.v[k] = q[k];
    return h;
}
// LDS records (16-byte aligned, klein_mfma_kernel rec_lds): four 16-byte reads + one
__device__ __forceinline__ QHead load_head(lds_cdptr q) {
    typedef double d2v __attribute__((ext_vector_type(2)));
    using lds_d2p = const __attribute__((address_space(3))) d2v*;
    QHead h;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const d2v t = ((lds_d2p)q)[k];
        h.v[2 * k] = t[0];
        h.v[2 * k + 1] = t[1];
    }
    h.v[8] = q[8];
    return h;
}

template <int NT, bool CERT, typename TP, typename QP>
__device__ __forceinline__ double sample_z_wide(double mu, double u, const QHead& h, QP q,
                                                int kind, int precision, bool linear_probs,
                                                bool want_log, TP etab, double& log_norm, double dmu) {
    const double sig = h.v[0], is = h.v[1];
    const double c = rint(mu);
    const double m = mu - c;
    double S, base, a, b;
    if (kind == kSzCapped) {
        S = q[kSzS + kSzDeg];
        base = q[kSzB + kSzDeg];
#pragma unroll
        for (int k = kSzDeg - 1; k >= 0; --k) {
            S = fma(S, m, q[kSzS + k]);
            base = fma(base, m, q[kSzB + k]);
        }
        a = -500.0;
        b = 500.0;
    } else {
        S = h.v[7];
        base = h.v[8];
        a = floor(mu - h.v[6]) - c;
        b = ceil(mu + h.v[6]) - c;
    }
    const double target = u * S;
    const float arg = fminf(fmaxf((float)((target + base) * h.v[4]), -1.0f + 0x1p-24f),
                            1.0f - 0x1p-24f);
    const float xg = fmaf((float)h.v[5], erfinvf(arg), (float)m);
    double kd = fmin(fmax((double)ceilf(xg - 0.5f), a), b);
    double fk;
    double Ck = em_C_rel<NT>(kd, m, sig, is, etab, base, fk);
#pragma nounroll
    for (int it = 0; it < 64 && Ck <= target && kd < b; ++it) {  // move up
        kd += 1.0;
        fk = gauss_tab(kd, m, is, etab);
        Ck += fk;
    }
#pragma nounroll
    for (int it = 0; it < 64 && kd > a && Ck - fk > target; ++it) {  // move down
        Ck -= fk;
        kd -= 1.0;
        fk = gauss_tab(kd, m, is, etab);
    }
    const double margin = fmin(Ck - target, kd > a ? target - (Ck - fk) : target);
    if constexpr (CERT) {
        // certificate: clear of the boundaries by the 0.6 dmu / s they can move;
        // a capped window is c +- 500 for every mean within dmu; the closed
        // window's ends carry < 1e-18 S (tails beyond +-9 s).  Not covered: the
        // decision as a guess, flagged by log_norm = NaN
        if (!(Ck > target)) return __builtin_nan("");
        if (!(margin > fma(0.6 * dmu, is, 1e-12) * S) || (kind == kSzCapped && !(fabs(m) + 1.01 * dmu < 0.5))) {
            log_norm = __builtin_nan("");
            return c + kd;
        }
    } else if (!(margin > 1e-12 * S) || !(Ck > target)) {
        // too close to call in fp64 (margin below 1e-12 S): sample_z_coord
        // finishes it with the exact table walk
        return __builtin_nan("");
    }
    log_norm = want_log ? log(S) : 0.0;
    return c + kd;
}

// Polynomial sum_k c[k] x^k by Estrin's scheme: depth ceil(log2 N) + 1 dependent
// FMAs instead of Horner's N - 1 (the capped decision is latency-bound).
template <int N>
__device__ __forceinline__ double poly_estrin(const double (&c)[N], double x) {
    double p[N];
#pragma unroll
    for (int k = 0; k < N; ++k) p[k] = c[k];
    int n = N;
    double xp = x;
#pragma unroll
    for (int lvl = 0; lvl < 6; ++lvl) {
        if (n > 1) {
#pragma unroll
            for (int j = 0; j < (n + 1) / 2; ++j) p[j] = 2 * j + 1 < n ? fma(p[2 * j + 1], xp, p[2 * j]) : p[2 * j];
            n = (n + 1) / 2;
            xp = xp * xp;
        }
    }
    return p[0];
}

// Polynomial coefficients of the capped decision (below), in constant memory and
// read through a pointer the compiler cannot prove invariant: inside the rolled
// coordinate loop of klein_mfma_kernel they are then scalar loads per coordinate
// instead of ~36 fp64 constants hoisted into VGPRs for the whole loop (with a copy
// before every fmac).
//   [0, 11)  erf(y)/y as a polynomial in z = y^2 on [0, 1] (Chebyshev fit; 4.5e-15 rel. of libm)
//   [11, 23) e^{-z} on [0, 1] (2.6e-15 rel.)
//   [23, 36) erfinv(v) = v R(v^2), |v| <= 0.849 (relative error 3e-8)
__device__ __constant__ double kCapCoef[36] = {
    1.1283791670955137, -0.3761263890318955, 0.11283791670856351, -0.0268661706101513, 0.005223977272142491,
    -0.000854830863419428, 0.00012054761075042809, -1.491439328403532e-05, 1.6319831426837587e-06,
    -1.5234934784514681e-07, 9.527703833862884e-09,
    0.9999999999999993, -0.9999999999999447, 0.4999999999972167, -0.16666666661556404, 0.04166666619559115,
    -0.008333330756823971, 0.0013888798425041814, -0.00019839153700921557, 2.4768196009077585e-05,
    -2.72048331078728e-06, 2.5149219471527703e-07, -1.5159419884388667e-08,
    0.8862269447150851, 0.23200895985592382, 0.1278390124627034, 0.07920907048159789, 0.16780265291085433,
    -0.8188084361376584, 4.787814391235978, -17.187235185827564, 42.14891487326897, -68.64189227692192,
    71.76515059941498, -43.593212219926436, 11.853485934431038};
constexpr int kCapE = 0, kCapG = 11, kCapRI = 23;
// kCapCoef[kCapRI ..] as compile-time constants (LGS_CAP_IMM)
constexpr double kCapRIImm[13] = {0.8862269447150851, 0.23200895985592382, 0.1278390124627034,
                                  0.07920907048159789, 0.16780265291085433, -0.8188084361376584,
                                  4.787814391235978, -17.187235185827564, 42.14891487326897,
                                  -68.64189227692192, 71.76515059941498, -43.593212219926436,
                                  11.853485934431038};
__device__ __forceinline__ cdptr cap_coef() {
    cdptr p = (cdptr)kCapCoef;
    asm volatile("" : "+s"(p));
    return p;
}
// Coefficients in SGPRs: Estrin's first level (both operands constants) costs a
// VGPR copy per pair; a two-way Horner split (even and odd coefficients as two
// interleaved Horner chains in x^2, each FMA with its scalar coefficient as the
// addend) needs no copies at about half Horner's depth.  LGS_CAP_ESTRIN: Estrin.
template <int N>
__device__ __forceinline__ double poly_h2(const double* c, double x);
template <int N>
__device__ __forceinline__ double poly_estrin_p(cdptr cf, double x) {
    double c[N];
#pragma unroll
    for (int k = 0; k < N; ++k) c[k] = cf[k];
    return poly_h2<N>(c, x);
}
// the coefficients already in (scalar) registers
template <int N>
__device__ __forceinline__ double poly_h2(const double* c, double x) {
#ifdef LGS_CAP_ESTRIN
    double cc[N];
#pragma unroll
    for (int k = 0; k < N; ++k) cc[k] = c[k];
    return poly_estrin(cc, x);
#else
    // v_fma_f64 with the scalar coefficient as the addend, written out: left to
    // itself the compiler picks v_fmac_f64 and copies the coefficient into the
    // accumulator register first
    auto fma_s = [](double a, double b, double sc) {
        double r;
        asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(sc));
        return r;
    };
    const double x2 = x * x;
    constexpr int NE = (N + 1) / 2, NO = N / 2;  // c[0], c[2], ... and c[1], c[3], ...
    double pe = c[2 * (NE - 1)], po = c[2 * (NO - 1) + 1];
#pragma unroll
    for (int k = NE - 2; k >= 0; --k) pe = fma_s(pe, x2, c[2 * k]);
#pragma unroll
    for (int k = NO - 2; k >= 0; --k) po = fma_s(po, x2, c[2 * k + 1]);
    return fma(po, x, pe);
#endif
}

// C(k) - base of a capped window with sigma >= 360 (Euler-Maclaurin with 3 terms,
// as em_P_tab<3>), erf / exp from fitted polynomials in Estrin form; fk = f(k).
__device__ __forceinline__ double capped_C(double kd, double m, double sig, double is, double base, double& fk,
                                           cdptr cf) {
    const double t = (kd - m) * is;
    const double t2 = t * t;
    const double z = 0.5 * t2;  // y^2, y = t / sqrt 2
    const double erf_y = (t * kInvSqrt2) * poly_estrin_p<11>(cf + kCapE, z);
    fk = poly_estrin_p<12>(cf + kCapG, z);
    // sum_m c_m He_{2m+1}(t) / sigma^{2m+1}: He1 = t, He3 = t^3 - 3t, He5 = t^5 - 10t^3 + 15t
    const double is2 = is * is;
    const double he3 = t * (t2 - 3.0);
    const double he5 = t * fma(t2, t2 - 10.0, 15.0);
    const double res = is * fma(is2, fma(is2 * (1.0 / 30240.0), he5, (-1.0 / 720.0) * he3), (1.0 / 12.0) * t);
    return fma(-res, fk, sig * kSqrtHalfPi * erf_y) + 0.5 * fk - base;
}

// The capped kind with sigma >= 360 (q[7] == 1: NTRU / q-ary bases' large-sigma
// coordinates), streamlined for latency -- the Klein kernels' per-coordinate
// dependency chain runs through it: the quantile guess from a fixed fp64 erfinv
// polynomial (|v| <= 0.849, relative error 3e-8; no branches, unlike erfinvf),
// the series erf / exp (PolyErf), and the +-1 walk only behind a wave-uniform test
// (the guess is off by one for ~4e-5 of the lanes).  Same decision rule, margins
// and certificate as sample_z_wide.
// The capped decision by evaluating C(k) at the guess (+-1 walk behind a
// wave-uniform test): the waves where some lane's quantile decision is not
// certain (sample_z_capped).  Out of line: its registers stay out of the Klein
// kernels' rolled near field, which runs it for ~0.1 % of the waves.
// (Both results come back in registers: a reference parameter of a call lives in
// the caller's scratch frame, a store per call that the next call waits for.)
struct SzPair {
    double z, ln;
};
template <bool CERT>
__device__ __noinline__ SzPair capped_slow(double c, double m, double sig, double is, double S, double base,
                                           double target, double xg, bool want_log, double dmu) {
    const cdptr cf = cap_coef();
    SzPair r = {__builtin_nan(""), 0.0};
    double kd = fmin(fmax(ceil(xg - 0.5), -500.0), 500.0);
    double fk;
    double Ck = capped_C(kd, m, sig, is, base, fk, cf);
    if (__builtin_amdgcn_ballot_w64(!(Ck > target) || (kd > -500.0 && Ck - fk > target)) != 0) {
#pragma nounroll
        for (int it = 0; it < 64 && Ck <= target && kd < 500.0; ++it) {  // move up
            kd += 1.0;
            fk = gauss_tab(kd, m, is, PolyErf{});
            Ck += fk;
        }
#pragma nounroll
        for (int it = 0; it < 64 && kd > -500.0 && Ck - fk > target; ++it) {  // move down
            Ck -= fk;
            kd -= 1.0;
            fk = gauss_tab(kd, m, is, PolyErf{});
        }
    }
    const double margin = fmin(Ck - target, kd > -500.0 ? target - (Ck - fk) : target);
    if constexpr (CERT) {
        if (!(Ck > target)) return r;
        if (!(margin > fma(0.6 * dmu, is, 1e-12) * S) || !(fabs(m) + 1.01 * dmu < 0.5)) {
            r.z = c + kd;
            r.ln = __builtin_nan("");
            return r;
        }
    } else if (!(margin > 1e-12 * S) || !(Ck > target)) {
        return r;
    }
    r.z = c + kd;
    r.ln = want_log ? log(S) : 0.0;
    return r;
}

#ifdef LGS_DIAG_CAPQ
__device__ unsigned long long lgs_diag_capq[8];
#endif
// The erfinv coefficients kCapCoef[kCapRI..] loaded into scalar registers ahead of
// the decision (load_cap_ri, at the top of a coordinate's step: the scalar-memory
// round trip then overlaps the record reads instead of sitting on the chain).
struct CapRI {
    double c[13];
};
__device__ __forceinline__ CapRI load_cap_ri() {
    const cdptr cf = cap_coef();
    CapRI r;
#pragma unroll
    for (int k = 0; k < 13; ++k) r.c[k] = cf[kCapRI + k];
#pragma unroll
    for (int k = 0; k < 13; ++k) asm volatile("" : "+s"(r.c[k]));
    return r;
}
// ln(x), x > 0 normal, with its constants through scalar registers (re-materialised
// where used: ocml's log coefficients were hoisted out of the Wang-Ling Klein
// near-field loop, spilled, and reloaded per coordinate behind vmcnt waits that also
// waited for the loop's stores).  x = 2^e m, m in [sqrt(1/2), sqrt(2)),
// ln m = 2 atanh(s), s = (m - 1) / (m + 1), |s| <= 0.1716: the series through s^25
// (truncation < 1e-19 relative), e ln2 in two parts (fdlibm's split, e ln2_hi exact).
// Within 1.8 ulp over [2^-1000, 2^1000] and near 1 (host replica against 40-digit
// decimal ln); the Wang-Ling weight bounds allow 1e-12 (1 + |ln|) per term.
__device__ __forceinline__ double ln_fast(double x) {
    int e;
    double m = frexp(x, &e);  // [1/2, 1)
    const bool lo = m < 0.70710678118654752440;
    m = lo ? 2.0 * m : m;
    e = lo ? e - 1 : e;
    const double s = (m - 1.0) / (m + 1.0);
    const double s2 = s * s;
    double p = 2.0 / 25.0;
    asm volatile("" : "+s"(p));
#pragma unroll
    for (int k = 11; k >= 1; --k) {
        double ck = 2.0 / (2.0 * k + 1.0);
        asm volatile("" : "+s"(ck));
        p = fma(p, s2, ck);
    }
    // p = 2/3 + 2/5 s^2 + ... + 2/25 s^22, so 2 s + s^3 p is the series through s^25
    const double lnm = fma(s * s2, p, 2.0 * s);
    double h = 6.93147180369123816490e-01, l = 1.90821492927058770002e-10;
    asm volatile("" : "+s"(h), "+s"(l));
    const double ed = (double)e;
    return fma(ed, h, fma(ed, l, lnm));
}

template <bool CERT, typename QP>
__device__ __forceinline__ double sample_z_capped(double mu, double u, const QHead& h, QP q, bool want_log,
                                                  double& log_norm, double dmu, const CapRI* ri = nullptr) {
    const double sig = h.v[0], is = h.v[1];
    const double c = rint(mu);
    const double m = mu - c;
    double cS[kSzDeg + 1], cB[kSzDeg + 1];
#pragma unroll
    for (int k = 0; k <= kSzDeg; ++k) {
        cS[k] = q[kSzS + k];
        cB[k] = q[kSzB + k];
    }
    const double S = poly_estrin(cS, m), base = poly_estrin(cB, m);
    const double target = u * S;
    // continuous quantile x = m + sigma sqrt(2) erfinv(v): erfinv(v) = v R(v^2)
    const cdptr cf = cap_coef();
    const double v = fmin(fmax((target + base) * h.v[4], -0.8485), 0.8485);
#ifdef LGS_CAP_IMM
    // the erfinv coefficients as scalar immediates (s_mov) at the use: no scalar-memory
    // round trip on the decision's dependency chain
    CapRI rim;
#pragma unroll
    for (int k = 0; k < 13; ++k) {
        rim.c[k] = kCapRIImm[k];
        asm volatile("" : "+s"(rim.c[k]));
    }
    (void)cf;
    const double xg = fma(h.v[5] * v, poly_h2<13>(rim.c, v * v), m);
#else
    const double xg = fma(h.v[5] * v, ri ? poly_h2<13>(ri->c, v * v) : poly_estrin_p<13>(cf + kCapRI, v * v), m);
#endif
#ifdef LGS_DIAG_CAP_GUESS  // diagnostic builds only (NOT bit-exact): cost probe, decision = the guess
    return c + fmin(fmax(ceil(xg - 0.5), -500.0), 500.0);
#endif
#ifndef LGS_CAP_NO_QUANTILE
    // Decision from the quantile alone, without evaluating C(k): with the window
    // sums C(k) of this kind (sigma >= 360), C(k) + base = sc erf(t(y_k) / sqrt 2)
    // at y_k = k + 1/2 + (k - m) / (24 sigma^2) to within 4e-11 units of y
    // (mpmath over sigma in [360, 1e10], every 7th k, tools/capped_quantile_check.py),
    // so C(k) > u S  <=>  k > xs = xg - 1/2 - (xg - m) / (24 sigma^2), and the decision
    // is floor(xs) + 1 whenever xs is farther from an integer than xs's error:
    // the erfinv polynomial's 2.93e-8 relative (|xg - m| <= 501.5), the reference's
    // fp64 cumsum within 1e-12 S (2.7e-9 units: f >= 0.379 over the window), fp64
    // rounding (< 1e-11 units), and for certified decisions a mean shift of up to
    // dmu (the boundary moves <= 0.6 dmu S / (sigma f) <= 4.5 dmu units, the
    // margin rule below in x units).  The rest (~3e-5 of the draws) go on below.
    {
        const double xs = fma((xg - m) * (-1.0 / 24.0), is * is, xg - 0.5);
        const double fl = floor(xs);
        // (the constant through a scalar register: hoisted into a VGPR pair out of the
        // near-field loop, the compiler spilled it, and its reload's vmcnt(0) waited for
        // every coordinate's stores)
        double t0 = 1e-8;
        asm volatile("" : "+s"(t0));
        const double tol = fma(2.94e-8, fabs(xg - m), CERT ? fma(4.5, dmu, t0) : t0);  // (plain: dmu < 0)
#ifdef LGS_DIAG_CAPQ  // diagnostic builds only: why the quantile decision falls through
        {
            const bool ca = !(xs - fl > tol && fl + 1.0 - xs > tol), cb = !(fl >= -501.0 && fl <= 499.0),
                       cc = !(fabs(v) < 0.848), cd = CERT && !(fabs(m) + 1.01 * dmu < 0.5);
            const unsigned long long b0 = __builtin_amdgcn_ballot_w64(true), b1 = __builtin_amdgcn_ballot_w64(ca),
                                     b2 = __builtin_amdgcn_ballot_w64(cb), b3 = __builtin_amdgcn_ballot_w64(cc),
                                     b4 = __builtin_amdgcn_ballot_w64(cd),
                                     b5 = __builtin_amdgcn_ballot_w64(ca || cb || cc || cd);
            if ((threadIdx.x & 63) == __builtin_ctzll(b0)) {
                atomicAdd(&lgs_diag_capq[0], (unsigned long long)__builtin_popcountll(b0));
                atomicAdd(&lgs_diag_capq[1], (unsigned long long)__builtin_popcountll(b1));
                atomicAdd(&lgs_diag_capq[2], (unsigned long long)__builtin_popcountll(b2));
                atomicAdd(&lgs_diag_capq[3], (unsigned long long)__builtin_popcountll(b3));
                atomicAdd(&lgs_diag_capq[4], (unsigned long long)__builtin_popcountll(b4));
                atomicAdd(&lgs_diag_capq[5], b5 != 0 ? 1ull : 0ull);
                atomicAdd(&lgs_diag_capq[6], 1ull);
            }
            atomicMax(&lgs_diag_capq[7], (unsigned long long)(dmu * 1e15));
        }
#endif
#ifdef LGS_CAP_BRANCHLESS  // every condition evaluated: straight-line compares, no exec-masked branch
        const bool fast = (xs - fl > tol) & (fl + 1.0 - xs > tol) & (fl >= -501.0) & (fl <= 499.0) &
                          (fabs(v) < 0.848) & (!CERT | (fabs(m) + 1.01 * dmu < 0.5));
#else
        const bool fast = xs - fl > tol && fl + 1.0 - xs > tol && fl >= -501.0 && fl <= 499.0 &&
                          fabs(v) < 0.848 && (!CERT || fabs(m) + 1.01 * dmu < 0.5);
#endif
        // a wave-uniform branch: the evaluation below must not be if-converted into
        // straight-line code that every wave runs
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(!fast) == 0, 1)) {
#ifndef LGS_LN_OCML  // (Wang-Ling Klein 4.84 -> 4.11 ms per 2^18 C3 samples, profiles/r04ah_*)
            log_norm = want_log ? ln_fast(S) : 0.0;
#else
            log_norm = want_log ? log(S) : 0.0;
#endif
            return c + (fl + 1.0);
        }
    }
#endif
    const SzPair r = capped_slow<CERT>(c, m, sig, is, S, base, target, xg, want_log, dmu);
    log_norm = r.ln;
    return r.z;
}

// Both window ends evaluated per draw (kinds without precomputed normalisers);
// out of line: its two concurrent erf evaluations would otherwise set the
// register footprint of sample_z_coord.
template <typename TP>
__device__ __noinline__ SampleZOut sample_z_generic(double mu, double sig, int precision,
                                                    bool linear_probs, double u, bool want_log,
                                                    TP etab, double dmu) {
    int64_t lo, hi;
    support_window(mu, sig, precision, lo, hi);
    return sig < 50.0 ? sample_z_em_tab<6>(mu, sig, precision, linear_probs, u, want_log, lo, hi, etab, dmu)
                      : sample_z_em_tab<3>(mu, sig, precision, linear_probs, u, want_log, lo, hi, etab, dmu);
}

// A wave-uniform pointer passed to a non-inlined function arrives in VGPRs;
// readfirstlane makes it scalar so its loads are s_load into SGPRs.
template <typename T>
__device__ __forceinline__ const T* uniform_ptr(const T* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (const T*)(((uint64_t)hi << 32) | lo);
}

// Per-coordinate constants arrive either as a constant-address-space pointer
// (made scalar inside the callee) or as an LDS pointer (records staged per panel).
__device__ __forceinline__ cdptr uniformize(cdptr p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (cdptr)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ lds_cdptr uniformize(lds_cdptr p) { return p; }
__device__ __forceinline__ gdptr uniformize(gdptr p) { return p; }  // (divergent callers)

// The per-coordinate decision proper is a leaf function: it makes no calls, so
// it needs no frame (a non-leaf callee saves its return address through a
// scratch store and reload on every call).  The rare cases it does not
// handle -- small-kind windows of more than 4 points, the generic kind and wide
// decisions within 1e-12 S of a boundary -- return NaN, and sample_z_coord
// below finishes them out of line.
template <bool CERT, typename TP, typename QP>
__device__ __forceinline__ double sample_z_coord_body(double mu, double u, QP qin, int precision,
                                                      bool linear_probs, bool want_log, TP etab,
                                                      double& log_norm, double dmu) {
    const QP q = uniformize(qin);  // all lanes are on the same coordinate
    const QHead qh = load_head(q);
    const int kind = (int)qh.v[2];
    const double sig = qh.v[0];
    if (kind == kSzSmall) {
        const double lo = floor(mu - qh.v[6]);
        const double hi = ceil(mu + qh.v[6]);
        if (hi - lo > 3.0) return __builtin_nan("");
        const double is = qh.v[1];
        constexpr bool cert = CERT;
        // window ends: checked when the points they can add or drop may carry more
        // than 2^-60 of the mass (q[7] = 1, host); below that such a point only
        // matters for u < 2^-60, i.e. u = 0 (q[7] = 0.5), and not at all when its
        // probability is exactly 0 (q[7] = 0).  Not covered: the decision as a
        // guess, log_norm = NaN
        const bool doubt =
            cert && (qh.v[7] == 1.0 ? !ends_stable(mu, qh.v[6], dmu) : (qh.v[7] != 0.0 && u == 0.0));
        double e[4];
        double emax = -INFINITY, e2 = -INFINITY, kmax = lo;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double t = ((lo + (double)k) - mu) * is;
            e[k] = lo + (double)k <= hi ? -0.5 * (t * t) : -INFINITY;
            const bool top = e[k] > emax;
            e2 = top ? emax : fmax(e2, e[k]);
            kmax = top ? lo + (double)k : kmax;
            emax = top ? e[k] : emax;
        }
        // one point outweighs every other by more than e^745.2: the others are
        // exactly 0 in fp64 (as in the general loop below), so the decision is that
        // point for every u (NTRU's sigma_i ~ 1e-3 coordinates, 2- and 3-point
        // windows) -- certified when the gap, moving by at most (hi - lo) / s^2 per
        // unit of mean, stays above 745.2 within dmu
        const double gap = emax - e2;
        if (gap > 745.2 && !(linear_probs && emax < -745.2)) {
            log_norm = (doubt || (cert && !(gap - 745.2 > 1.01 * dmu * (hi - lo) * (is * is) + 1e-12 * gap)))
                           ? __builtin_nan("")
                           : (want_log ? emax : 0.0);
            return kmax;
        }
        if (linear_probs && emax < -745.2) {
            log_norm = cert ? __builtin_nan("") : -INFINITY;
            return rint(mu);
        }
        double w[4];
        double Ssum = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double x = e[k] - emax;
            w[k] = x == 0.0 ? 1.0 : (x < -745.2 ? 0.0 : exp(x));
            Ssum += w[k];
        }
        const double target = u * Ssum;
        double C = 0.0, z = hi, Cp = 0.0, Cz = Ssum;
        bool found = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double Cn = C + w[k];
            if (!found && lo + (double)k <= hi && Cn > target) {
                z = lo + (double)k;
                found = true;
                Cp = C;
                Cz = Cn;
            }
            C = Cn;
        }
        log_norm = want_log ? emax + log(Ssum) : 0.0;
        if (cert) {
            // boundary odds move by at most e^{(hi - lo) dmu / s^2}
            const double E = odds_factor((hi - lo) * dmu * (is * is));
            if (doubt || (linear_probs && emax < -700.0) || (z > lo && !boundary_clear(target, Cp, Ssum, E)) ||
                (z < hi && !boundary_clear(target, Cz, Ssum, E)))
                log_norm = __builtin_nan("");
        }
        return z;
    }
    if (kind == kSzGeneric) return __builtin_nan("");
#ifndef LGS_NO_CAPPED_POLY
    if (kind == kSzCapped && qh.v[7] == 1.0)  // sigma >= 360 (host): series erf / exp
        return sample_z_capped<CERT>(mu, u, qh, q, want_log, log_norm, dmu);
#endif
    return sig < 50.0
               ? sample_z_wide<6, CERT>(mu, u, qh, q, kind, precision, linear_probs, want_log, etab, log_norm, dmu)
               : sample_z_wide<3, CERT>(mu, u, qh, q, kind, precision, linear_probs, want_log, etab, log_norm, dmu);
}

template <bool CERT, typename TP, typename QP>
LGS_SAMPLEZ_ATTR SzPair sample_z_coord_leaf(double mu, double u, QP q, int precision,
                                            bool linear_probs, bool want_log, TP etab, double dmu) {
    SzPair r;
    r.ln = 0.0;
    r.z = sample_z_coord_body<CERT>(mu, u, q, precision, linear_probs, want_log, etab, r.ln, dmu);
    return r;
}

template <typename TP>
__device__ __noinline__ double sample_z_coord_fallback(double mu, double u, double sig, int kind,
                                                       int precision, bool linear_probs,
                                                       bool want_log, TP etab, double& log_norm,
                                                       double dmu) {
    const SampleZOut o = kind == kSzGeneric
                             ? sample_z_generic(mu, sig, precision, linear_probs, u, want_log, etab, dmu)
                             : sample_z_table(mu, sig, precision, linear_probs, u, want_log, dmu);
    log_norm = o.log_norm;
    return o.z == kAmbZ ? kAmbiguous : (double)o.z;
}

// SampleZ for one coordinate from its precomputed constants (kinds in lgs_kernels.h).
// dmu >= 0: certified decision (see "certified decisions" above; kAmbiguous when
// not covered); dmu < 0: plain decision at mu.
template <typename TP, typename QP>
__device__ __forceinline__ double sample_z_coord(double mu, double u, QP q, int precision,
                                                 bool linear_probs, bool want_log, TP etab,
                                                 double& log_norm, double dmu) {
    const SzPair r = dmu >= 0.0
                         ? sample_z_coord_leaf<true>(mu, u, q, precision, linear_probs, want_log, etab, dmu)
                         : sample_z_coord_leaf<false>(mu, u, q, precision, linear_probs, want_log, etab, dmu);
    double z = r.z;
    log_norm = r.ln;
    if (dmu >= 0.0 && !__builtin_isnan(z) && __builtin_isnan(r.ln)) return kAmbiguous;
    if (__builtin_isnan(z))
        z = sample_z_coord_fallback(mu, u, q[0], (int)q[2], precision, linear_probs, want_log, etab,
                                    log_norm, dmu);
    return z;
}
// The capped kind with sigma >= 360 alone (klein_mfma_kernel dispatches on the
// kind itself): a small leaf, no kind dispatch inside (inlined into the rolled
// near field, LGS_CAPPED_INLINE).
template <bool CERT, typename QP>
#ifdef LGS_CAPPED_INLINE
__device__ __forceinline__
#else
__device__ __noinline__
#endif
SzPair sample_z_capped_leaf(double mu, double u, QP q, bool want_log, double dmu) {
    const QP qu = uniformize(q);
    const QHead qh = load_head(qu);
    SzPair r;
    r.ln = 0.0;
    r.z = sample_z_capped<CERT>(mu, u, qh, qu, want_log, r.ln, dmu);
    return r;
}

// The NaN conventions of a leaf's result resolved (fallback decision; CERT: guess
// flagged in amb).
template <bool CERT, typename TP, typename QP>
__device__ __forceinline__ double sz_finish(SzPair r, double mu, double u, QP q, int precision,
                                            bool linear_probs, bool want_log, TP etab,
                                            double& log_norm, double dmu, bool& amb) {
    double z = r.z;
    log_norm = r.ln;
    amb = false;
    if (__builtin_isnan(z)) {
        z = sample_z_coord_fallback(mu, u, q[0], (int)q[2], precision, linear_probs, want_log, etab,
                                    log_norm, CERT ? dmu : -1.0);
        if (CERT && z == kAmbiguous) {
            z = rint(mu);
            amb = true;
        }
    } else if (CERT && __builtin_isnan(r.ln)) {
        amb = true;
    }
    if (amb) log_norm = 0.0;
    return z;
}

// Conditional mean of coordinate i in the reference's order (klein.py:191-195:
// j ascending, separate multiply and add -- the file is built with
// -ffp-contract=off), from the sample's own stored coefficients z_j, j > i.
// Used for the rare decisions the certificate does not cover.
template <typename ZT>
__device__ __noinline__ double mu_exact_col(const double* __restrict__ R, const ZT* __restrict__ Zp,
                                            size_t ldz, int i, int d, double cp, double rii) {
    const double* __restrict__ Ri = R + (size_t)i * d;
    double cs = 0.0;
    for (int j = i + 1; j < d; ++j) cs = cs + Ri[j] * (double)Zp[(size_t)j * ldz];
    return (cp - cs) / rii;
}

}  // namespace lgs
