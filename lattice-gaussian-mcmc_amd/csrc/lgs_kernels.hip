// lgs_kernels.hip -- HIP/CDNA4 kernels of the Klein / IMHK hot path (gfx950).
//
//   klein_exact_kernel  Klein randomized nearest plane, reference arithmetic order
//                       (klein.py:181-220: sequential j-ascending unfused fp64 sums),
//                       one chain (sample) per lane.
//   klein_panel_kernel  Same sampler, blocked: PB rows per panel, far-field
//                       contributions left-looking from the coefficient store
//                       (one coalesced load feeds PB FMAs), near field right-looking
//                       in registers.  Default (fast) mode.
//   imhk_accept_kernel  Metropolis test of imhk.py:141-177 over a block of steps,
//                       one chain per lane (proposals are independent of the state).
//   bz_gemm_kernel      v = B z for a batch (klein.py:218), fp64 MFMA 16x16x4.
//   moments / gathers / transpose helpers.
//
// Coefficient store layout: Z[coord][lane] ("coordinate-major", ld = ldz) so that
// every access of the sampler is a 64-lane coalesced row segment.
//
// Compiled with -ffp-contract=off (see lgs_device.h).
#include <hip/hip_runtime.h>

#include <type_traits>
#include <stdint.h>

// The rolled near field (default) decides the capped kind inline (one copy in the
// loop body); the unrolled one (LGS_NEAR_UNROLLED) calls it as a leaf.
#if !defined(LGS_NEAR_UNROLLED) && !defined(LGS_CAPPED_CALL) && !defined(LGS_CAPPED_INLINE)
#define LGS_CAPPED_INLINE
#endif
#include "lgs_device.h"
#include "lgs_kernels.h"

namespace lgs {

typedef unsigned int v4u_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void lane_counter(const KleinArgs& a, int64_t p, uint32_t& chain,
                                             uint32_t& step) {
    if (a.counter_mode == 0) {
        const uint64_t s = a.base + (uint64_t)p;
        chain = (uint32_t)s;
        step = (uint32_t)(s >> 32);
    } else {
        chain = a.chain0 + (uint32_t)(p / a.nt);
        step = a.step0 + (uint32_t)(p % a.nt);
    }
}

// Reference-mode importance weight term of one coordinate (imhk.py:102-124):
// log_gaussian_weight(Bz) - compute_log_density(Bz), with ||Bz - c||^2 =
// sum_i (R_ii (z_i - mu_i))^2.
__device__ __forceinline__ double ref_weight(double zi, double mu, double ros, double isr, double lterm) {
    const double res = zi - mu;
    const double ta = res * ros;
    const double tq = res * isr;
    return (-0.5 * (ta * ta)) - (-0.5 * (tq * tq) - lterm);
}

// Certificate bound dmu >= |mu - mu_ref| of coordinate i (lgs_device.h "certified
// decisions"; constants from lgs_set_basis), z1 = sum_{j>i} |z_j| of the sample.
__device__ __forceinline__ double cert_dmu(double ca, double cb, double z1, double mu) {
#ifdef LGS_DIAG_NO_CERT  // diagnostic builds only: cost probe of the certificate (NOT bit-exact)
    return -1.0;
#endif
    return fma(cb, z1, ca) + 6e-16 * fabs(mu);
}

// Wang-Ling weight bounds (certified decisions, blocked kernels).  A coordinate's
// term is the window's log normaliser ln(mu) = log sum_k exp(-(k - mu)^2 / (2 s^2))
// (imhk.py:102-124 via the SampleZ table of klein.py:129-139), evaluated at the
// blocked-order mean; the reference evaluates it at mu_ref, |mu - mu_ref| <= dmu
// (the certificate).  d ln / d mu = E_w[k - mu] / s^2, so with every window point
// within hw of mu:  |ln(mu) - ln(mu_ref)| <= (hw + dmu) dmu / s^2.  The window is
// the same at both means (certified decisions check its ends), and 1e-12 (1 + |ln|)
// covers the two evaluations' rounding and the rare table-walk path (its sum of
// <= 1001 terms against the closed / fitted normaliser).  One dominant point c
// (ln = -(c - mu)^2 / (2 s^2), the same c at both means): the exact difference
// (d1 + dmu / 2) dmu / s^2, d1 = |c - mu|, plus 1e-15 (1 + |ln|) for the three
// roundings.  The sum over coordinates (same order in both kernels) adds at most
// 2.5 u (d + 1) sum |terms| (wl_bound_sum).
__device__ __forceinline__ double wl_bound_generic(double ln, double is, double hw, double dmu) {
    return (hw + dmu) * (is * is) * dmu + 1e-12 * (1.0 + fabs(ln));
}
__device__ __forceinline__ double wl_bound_dominant(double emax, double is2, double d1, double dmu) {
    return is2 * dmu * (d1 + 0.5 * dmu) + 1e-15 * (1.0 + fabs(emax));
}
__device__ __forceinline__ double wl_bound_sum(double eb, double tb, int d) {
    return eb + 2.8e-16 * (double)(d + 1) * tb;
}
// half-width + 1 of the support window (klein.py:113-128): rf sigma, capped at 500
__device__ __forceinline__ double wl_window_hw(double rf_sigma) { return fmin(rf_sigma, 500.0) + 1.0; }
// per-sample bound out, and the wave's largest one into the context's running maximum
__device__ __forceinline__ void wl_bound_store(const KleinArgs& a, int64_t p, double e) {
    if (a.LWE) a.LWE[p] = e;
    if (a.emax) atomicMax(a.emax, (unsigned long long)__double_as_longlong(e));
}

// One coordinate's decision + weight bookkeeping, shared by both samplers.
// dmu >= 0: certified decision (kAmbiguous when the reference-order mean could
// decide otherwise; lw is then untouched); dmu < 0: decide at mu.
// WL: eb / tb accumulate the term's bound (wl_bound_generic) and |term|.
template <bool WL, typename TP>
__device__ __forceinline__ double decide_coord(const KleinArgs& a, int i, double mu,
                                               CoordStream& rs, double& lw, unsigned int& flags,
                                               TP etab, double dmu, double& eb, double& tb) {
    double zi;
    if (!isfinite(mu)) {
        flags |= kFlagNonFinite;
        return 0.0;
    }
    const double s = a.szc ? cst(a.szc)[(size_t)i * kSzcStride] : cst(a.sig)[i];
#ifdef LGS_DIAG_NO_SAMPLEZ
    if (true) {  // diagnostic build: SampleZ replaced by rounding
        zi = rint(mu + rs.u((uint32_t)(a.d - 1 - i)) * 1e-300);
    } else
#endif
#ifdef LGS_DIAG_SZ_KIND_ONLY
    if (a.szc && (int)cst(a.szc)[(size_t)i * kSzcStride + 2] != LGS_DIAG_SZ_KIND_ONLY) {
        zi = rint(mu + rs.u((uint32_t)(a.d - 1 - i)) * 1e-300);
    } else
#endif
    if (s == 0.0) {  // sigma_i < 1e-10: round, no draw (klein.py:201-204)
        zi = rint(mu);
        if (dmu >= 0.0 && !round_stable(mu, dmu)) return kAmbiguous;
    } else if (a.szc) {
        double ln;
        zi = sample_z_coord(mu, rs.u((uint32_t)(a.d - 1 - i)), cst(a.szc) + (size_t)i * kSzcStride,
                            a.precision, a.linear_probs != 0, WL, etab, ln, dmu);
        if (zi == kAmbiguous) return kAmbiguous;
        if (WL) {
            lw += ln;
            tb += fabs(ln);
            if (dmu >= 0.0)
                eb += wl_bound_generic(ln, cst(a.szc)[(size_t)i * kSzcStride + 1],
                                       wl_window_hw(cst(a.szc)[(size_t)i * kSzcStride + 6]), dmu);
        }
    } else {
        SampleZOut o = sample_z(mu, s, a.precision, a.linear_probs != 0,
                                rs.u((uint32_t)(a.d - 1 - i)), WL, a.etab, dmu);
        if (o.z == kAmbZ) return kAmbiguous;
        zi = (double)o.z;
        if (WL) {
            lw += o.log_norm;
            tb += fabs(o.log_norm);
            const double rf = s < 0.1 ? (double)(a.precision > 3 ? a.precision : 3) : (double)a.precision;
            if (dmu >= 0.0) eb += wl_bound_generic(o.log_norm, 1.0 / s, wl_window_hw(rf * s), dmu);
        }
    }
    if (!WL) lw += ref_weight(zi, mu, cst(a.ros)[i], cst(a.isr)[i], cst(a.lterm)[i]);
    return zi;
}

// A coordinate's Klein record (kRecStride doubles, staged in LDS per 32-row panel)
// read into registers as one batch of 16-byte LDS reads at the top of the
// coordinate's step, before anything branches on it: one LDS round trip per
// coordinate instead of one per use site (mean, kind, window, polynomials,
// weight terms, near-field coefficients), each behind the previous branch.
// (LGS_CAP_RI_PRE: the capped kind's erfinv coefficients come along as scalar loads;
// round 4: off by default -- without it, and with the Philox products as mul_lo /
// mul_hi pairs, the kernel spills 49 instead of 63 VGPRs and runs C2 / C3 / C4 / C5
// 4 / 2 / 3 / 3 % faster, outputs identical, profiles/r04ac_kbench_mulhi_noripre.log)
#ifdef LGS_REC_L2
constexpr int kRecHot = 46;  // (with the coarse panels' Cb, read in the batch instead of on its own)
#else
constexpr int kRecHot = 44;  // through the 15 near-field coefficients and the dispatch code
#endif
static_assert(kRecDisp < kRecHot && kRecRs + 15 <= kRecHot && kRecLterm < kRecHot, "hot record fields");
#ifdef LGS_REC_SMEM
// (experiment) the record read from the basis' record array in memory through a
// wave-uniform constant pointer at each use: scalar loads into SGPRs (no LDS reads, no
// 88 VGPRs holding wave-uniform values)
struct RecRegs {
    cdptr p;
    __device__ __forceinline__ double operator[](int k) const { return p[k]; }
};
#elif defined(LGS_REC_RS_SMEM)
// (experiment) the decision's fields from LDS as before, the 15 near-field coefficients
// (used last in the step) through scalar loads
struct RecRegs {
    double v[kRecHot];
    cdptr p;
    __device__ __forceinline__ double operator[](int k) const {
        return (k >= kRecRs && k < kRecRs + 15) ? p[k] : v[k];
    }
};
#else
struct RecRegs {
    double v[kRecHot];
#ifdef LGS_CAP_RI_PRE
    CapRI ri;
#endif
    __device__ __forceinline__ double operator[](int k) const { return v[k]; }
};
#endif
struct NoMid {
    __device__ __forceinline__ void operator()() const {}
};
#ifdef LGS_REC_SMEM
__device__ __forceinline__ RecRegs load_rec_g(cdptr grec) { return RecRegs{uniformize(grec)}; }
#else
template <typename MID = NoMid>
#ifdef LGS_REC_RS_SMEM
__device__ __forceinline__ RecRegs load_rec(lds_cdptr rec, cdptr gp, MID mid = MID{}) {
#else
__device__ __forceinline__ RecRegs load_rec(lds_cdptr rec, MID mid = MID{}) {
#endif
    typedef double d2v __attribute__((ext_vector_type(2)));
    using lds_d2p = const __attribute__((address_space(3))) d2v*;
    RecRegs r;
#ifdef LGS_REC_RS_SMEM
    static_assert(kRecRs % 2 == 0 && kRecDisp == kRecRs + 15 && kRecHot == kRecDisp + 1, "record layout");
#pragma unroll
    for (int k = 0; k < kRecHot / 2; ++k) {
        if (2 * k >= kRecRs && 2 * k + 1 < kRecRs + 15) continue;
        const d2v t = ((lds_d2p)rec)[k];
        r.v[2 * k] = t[0];
        r.v[2 * k + 1] = t[1];
    }
    r.p = uniformize(gp);
#else
#pragma unroll
    for (int k = 0; k < kRecHot / 2; ++k) {
        const d2v t = ((lds_d2p)rec)[k];
        r.v[2 * k] = t[0];
        r.v[2 * k + 1] = t[1];
    }
#endif
    mid();
#ifdef LGS_CAP_RI_PRE
    r.ri = load_cap_ri();
#endif
    // pinned here: left alone, the compiler sinks each read into the branch that
    // uses it (three round trips after the kind / window branches).
#if !defined(LGS_REC_NOPIN) && !defined(LGS_REC_L2) && defined(LGS_REC_PIN_BATCH)
    // (LGS_REC_PIN_BATCH: two asm statements over 22 registers each, one wait for the
    // batch instead of one s_waitcnt lgkmcnt(k) per register -- the allocator then
    // adds ~9 v_mov_b64 copies per step)
    static_assert(kRecHot == 44, "two pins of 22");
#define LGS_PIN22(o)                                                                                         \
    asm volatile("" : "+v"(r.v[o + 0]), "+v"(r.v[o + 1]), "+v"(r.v[o + 2]), "+v"(r.v[o + 3]), "+v"(r.v[o + 4]),   \
                 "+v"(r.v[o + 5]), "+v"(r.v[o + 6]), "+v"(r.v[o + 7]), "+v"(r.v[o + 8]), "+v"(r.v[o + 9]),        \
                 "+v"(r.v[o + 10]), "+v"(r.v[o + 11]), "+v"(r.v[o + 12]), "+v"(r.v[o + 13]), "+v"(r.v[o + 14]),   \
                 "+v"(r.v[o + 15]), "+v"(r.v[o + 16]), "+v"(r.v[o + 17]), "+v"(r.v[o + 18]), "+v"(r.v[o + 19]),   \
                 "+v"(r.v[o + 20]), "+v"(r.v[o + 21]))
    LGS_PIN22(0);
    LGS_PIN22(22);
#undef LGS_PIN22
#elif !defined(LGS_REC_NOPIN)
#pragma unroll
    for (int k = 0; k < kRecHot; ++k)
#ifdef LGS_REC_L2  // (Rs[1..14] not pinned: the first use waits for them)
        if (k <= kRecRs)
#elif defined(LGS_REC_RS_SMEM)
        if (k < kRecRs || k >= kRecRs + 14)
#endif
            asm volatile("" : "+v"(r.v[k]));
#endif
    return r;
}
#endif
#ifdef LGS_REC_L2
#define REC_CBC rr[kRecCbC]
#else
#define REC_CBC rec[kRecCbC]
#endif
struct RecView {  // q[k] of the SampleZ functions, served from the registers
    const RecRegs& r;
    __device__ __forceinline__ double operator[](int k) const { return r[k]; }
};

// decide_coord with the coordinate's record rec staged in LDS (klein_mfma_kernel,
// 32-row panels); rr: the record's registers (load_rec), rec for the rare paths.
// LIBM: the SampleZ path without per-coordinate constants (LGS_SAMPLEZ_LIBM); a
// separate kernel instantiation, so the default kernel carries one call path.
template <bool WL, bool CERT, bool LIBM, typename TP>
__device__ __forceinline__ double decide_coord_rec(const KleinArgs& a, int i, double mu,
                                                   lds_cdptr rec, const RecRegs& rr, CoordStream& rs, double& lw,
                                                   unsigned int& flags, TP etab, double dmu, bool& amb,
                                                   double& eb, double& tb) {
    double zi = 0.0;
    amb = false;
    if (!isfinite(mu)) {
        flags |= kFlagNonFinite;
        return 0.0;
    }
    QHead qh;
#pragma unroll
    for (int k = 0; k < 9; ++k) qh.v[k] = rr[k];
    const double s = qh.v[0];
#ifdef LGS_DIAG_NO_SAMPLEZ
    if (true) {
        zi = rint(mu + rs.u((uint32_t)(a.d - 1 - i)) * 1e-300);
    } else
#endif
#ifdef LGS_DIAG_SZ_KIND_ONLY
    if ((int)rec[2] != LGS_DIAG_SZ_KIND_ONLY) {
        zi = rint(mu + rs.u((uint32_t)(a.d - 1 - i)) * 1e-300);
    } else
#endif
#if defined(LGS_DISP_CODE) && defined(LGS_DISP_FIRST)
    // the capped sigma >= 360 kind tested first, on the host's dispatch code (scalar),
    // ahead of the sigma == 0 test (a vector compare and an exec-masked branch)
    if (!LIBM && __builtin_amdgcn_readfirstlane(__double2hiint(rr[kRecDisp])) == 0x3ff00000) {
        const double u = rs.u((uint32_t)(a.d - 1 - i));
        SzPair r;
        r.ln = 0.0;
        r.z = sample_z_capped<CERT>(mu, u, qh, RecView{rr}, WL, r.ln, dmu);
        double ln = 0.0;
        zi = sz_finish<CERT>(r, mu, u, rec, a.precision, a.linear_probs != 0, WL, etab, ln, dmu, amb);
        if (WL) {
            lw += ln;
            tb += fabs(ln);
            eb += amb ? 0.0 : wl_bound_generic(ln, qh.v[1], wl_window_hw(qh.v[6]), dmu);
        }
    } else
#endif
    // CERT: a decision not covered by the certificate is returned as a guess with
    // amb set and no weight term (the sub-panel's verification adds it); selects
    // instead of early returns keep the weight update branch-free (measured 13 vs
    // 44 spilled VGPRs)
    if (s == 0.0) {
        zi = rint(mu);
        amb = CERT && !round_stable(mu, dmu);
    } else if (LIBM) {  // LGS_SAMPLEZ_LIBM: generic path
        SampleZOut o = sample_z(mu, s, a.precision, a.linear_probs != 0,
                                rs.u((uint32_t)(a.d - 1 - i)), WL, a.etab, CERT ? dmu : -1.0);
        amb = CERT && o.z == kAmbZ;
        zi = amb ? rint(mu) : (double)o.z;
        if (WL) {
            const double ln = amb ? 0.0 : o.log_norm;
            lw += ln;
            tb += fabs(ln);
            eb += amb ? 0.0 : wl_bound_generic(ln, qh.v[1], wl_window_hw(qh.v[6]), dmu);
        }
    } else {
        // Inline one-dominant-point decision of the small kind (NTRU's sigma_i ~ 1e-3
        // coordinates), certified as in sample_z_coord_body: no call and no Philox
        // draw (the counter-addressed uniform is simply not generated: its value
        // cannot matter when every other window point, and any point the window's
        // ends could add, has probability exactly 0 -- rec[7] == 0)
        bool fast = false;
        double ln = 0.0;
        double ebf = 0.0;  // (WL) the fast decision's weight bound
        // the kind and its flag are the same in every lane: scalar branches
#ifdef LGS_DISP_CODE
        // the host's dispatch code (kRecDisp): one scalar read of its high word (0 for
        // 0.0, 0x3ff00000 for 1.0) instead of converting the kind and testing q[7]
        const int dsp = __builtin_amdgcn_readfirstlane(__double2hiint(rr[kRecDisp]));
        const bool small_fast = dsp == 0, capped1 = dsp == 0x3ff00000;
#else
        const int kind = __builtin_amdgcn_readfirstlane((int)qh.v[2]);
        const int q7 = __builtin_amdgcn_readfirstlane(qh.v[7] == 0.0 ? 0 : (qh.v[7] == 1.0 ? 1 : 2));
        const bool small_fast = kind == kSzSmall && q7 == 0, capped1 = kind == kSzCapped && q7 == 1;
#endif
        if (CERT && small_fast) {
            // the heaviest window point is rint(mu) (d1 = |mu - rint(mu)| < 1/2 unless a
            // tie, which fails the test); every other point lies >= 1 - d1 from mu, so
            // its log-weight is below the top one by >= is^2 (1 - 2 d1) / 2 -- a lower
            // bound of the gap the general path computes from the window's exponents
            const double is = qh.v[1], is2 = is * is;
            const double c = rint(mu), d1 = fabs(mu - c), t = d1 * is;
            const double emax = -0.5 * (t * t);
            const double gap = 0.5 * is2 * (1.0 - 2.0 * d1);
            const double hl = ceil(mu + qh.v[6]) - floor(mu - qh.v[6]);
            fast = gap > 745.2 && !(a.linear_probs && emax < -745.2) &&
                   gap - 745.2 > 1.01 * dmu * hl * is2 + 1e-12 * gap;
            zi = c;
            ln = emax;
            if (WL) ebf = wl_bound_dominant(emax, is2, d1, dmu);
        }
        if (!fast) {
            const double u = rs.u((uint32_t)(a.d - 1 - i));
            SzPair r;
#ifdef LGS_DIAG_NO_GENERIC  // diagnostic builds only: cost of the generic call sites (NOT bit-exact)
            if (capped1) {
                r = sample_z_capped_leaf<CERT>(mu, u, rec, WL, dmu);
                amb = CERT && (__builtin_isnan(r.z) || __builtin_isnan(r.ln));
                zi = __builtin_isnan(r.z) ? rint(mu) : r.z;
                ln = amb ? 0.0 : r.ln;
            } else {
                zi = rint(mu);
            }
            if (false)
#endif
            {
#ifndef LGS_NO_CAPPED_POLY
            if (capped1) {  // sigma >= 360: the streamlined capped decision
                r.ln = 0.0;
#ifdef LGS_CAP_RI_PRE
                r.z = sample_z_capped<CERT>(mu, u, qh, RecView{rr}, WL, r.ln, dmu, &rr.ri);
#else
                r.z = sample_z_capped<CERT>(mu, u, qh, RecView{rr}, WL, r.ln, dmu);
#endif
            } else
#endif
                r = sample_z_coord_leaf<CERT>(mu, u, rec, a.precision, a.linear_probs != 0, WL, etab, dmu);
            zi = sz_finish<CERT>(r, mu, u, rec, a.precision, a.linear_probs != 0, WL, etab, ln, dmu, amb);
            }
            if (WL) ebf = amb ? 0.0 : wl_bound_generic(ln, qh.v[1], wl_window_hw(qh.v[6]), dmu);
        }
        if (WL) {
            lw += ln;
            tb += fabs(ln);
            eb += ebf;
        }
    }
    if (!WL) {
        const double t = ref_weight(zi, mu, rr[kRecRos], rr[kRecIsr], rr[kRecLterm]);
        lw += amb ? 0.0 : t;
    }
    return zi;
}

// The rolled near field's running-sum update acc[k + 1] = fma(r, z, acc[k]) (k
// descending, in place).  Left to itself the compiler selects the two-address
// v_fmac_f64 (dst = addend): each result then lands in the register of acc[k], and
// the loop's back edge needs 15 v_mov_b64 per coordinate to shift the sums back.
// The three-address v_fma_f64 writes acc[k + 1]'s own register: no moves, the same
// fused operations (round 5: Klein 2.507 / 2.513 -> 2.443 / 2.456 ms per 2^18 C3
// samples, identical outputs, profiles/r05b_kb.log).  LGS_NEAR_FMA_PLAIN: fma().
__device__ __forceinline__ double fma_shift(double a, double b, double c) {
#ifndef LGS_NEAR_FMA_PLAIN
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return fma(a, b, c);
#endif
}

// decide_coord_rec for a coordinate of a sub-panel the host flagged all capped with
// sigma >= 360 (kRecSpec == 2: kind kSzCapped, q[7] == 1, sigma_i != 0): the same
// decision and weight bookkeeping without the per-coordinate kind dispatch (its
// vector -> scalar turnarounds sit on the near field's dependency chain).
template <bool WL, typename TP>
__device__ __forceinline__ double decide_capped_rec(const KleinArgs& a, int i, double mu, lds_cdptr rec,
                                                    const RecRegs& rr, CoordStream& rs, double& lw,
                                                    unsigned int& flags, TP etab, double dmu, bool& amb,
                                                    double& eb, double& tb) {
    amb = false;
    if (!isfinite(mu)) {
        flags |= kFlagNonFinite;
        return 0.0;
    }
    QHead qh;
#pragma unroll
    for (int k = 0; k < 9; ++k) qh.v[k] = rr[k];
    const double u = rs.u((uint32_t)(a.d - 1 - i));
    SzPair r;
    r.ln = 0.0;
    r.z = sample_z_capped<true>(mu, u, qh, RecView{rr}, WL, r.ln, dmu);
    double ln = 0.0;
    const double zi = sz_finish<true>(r, mu, u, rec, a.precision, a.linear_probs != 0, WL, etab, ln, dmu, amb);
    if (WL) {
        lw += ln;
        tb += fabs(ln);
        eb += amb ? 0.0 : wl_bound_generic(ln, qh.v[1], wl_window_hw(qh.v[6]), dmu);
    } else {
        const double t = ref_weight(zi, mu, rr[kRecRos], rr[kRecIsr], rr[kRecLterm]);
        lw += amb ? 0.0 : t;
    }
    return zi;
}

// z is an exact fp64 integer; int64 stores convert it, narrower stores flag
// values outside their range.
template <typename ZT>
__device__ __forceinline__ void store_z(ZT* Z, size_t off, double zi, unsigned int& flags) {
    if (sizeof(ZT) == 8) {
        Z[off] = (ZT)(int64_t)zi;
        return;
    }
    if (sizeof(ZT) == 4 && !(zi <= 2147483647.0 && zi >= -2147483648.0)) flags |= kFlagOverflow;
    if (sizeof(ZT) == 2 && !(zi <= 32767.0 && zi >= -32768.0)) flags |= kFlagOverflow16;
    Z[off] = (ZT)(int)fmin(fmax(zi, -2147483648.0), 2147483647.0);
}

// Stages the SampleZ erf/exp table in LDS (block-wide; call before any early return).
__device__ __forceinline__ lds_cdptr stage_etab(double* tab_lds, const double* __restrict__ etab) {
    if (etab)
        for (int k = threadIdx.x; k < 2 * (kErfTabLast + 1); k += blockDim.x) tab_lds[k] = etab[k];
    __syncthreads();
    return (lds_cdptr)tab_lds;
}

// A decision the certificate does not cover (rare; lanes diverge): the
// coordinate's mean in the reference's order from the sample's stored z_j (j > i,
// Zp = &Z[0][p]), then the plain decision at that mean with the same uniform.
// Out of line, with every input as a plain value.  Counted in *cnt.
struct Resolved {
    double z, ln, mu;
};
template <typename ZT>
__device__ __noinline__ Resolved resolve_decision(const double* __restrict__ R, const ZT* __restrict__ Zp,
                                                  size_t ldz, int i, int d, double cp, double rii,
                                                  const double* __restrict__ q, double s, double u,
                                                  int precision, bool linear, bool want_log,
                                                  const double* __restrict__ etab, unsigned int* cnt) {
    Resolved r;
    r.mu = mu_exact_col(R, Zp, ldz, i, d, cp, rii);
    r.ln = 0.0;
    r.z = 0.0;
    atomicAdd(cnt, 1u);
    if (!isfinite(r.mu)) return r;
    if (s == 0.0) {
        r.z = rint(r.mu);
    } else if (q) {
        r.z = sample_z_coord(r.mu, u, (gdptr)q, precision, linear, want_log, (gdptr)etab, r.ln, -1.0);
    } else {
        const SampleZOut o = sample_z(r.mu, s, precision, linear, u, want_log, etab);
        r.z = (double)o.z;
        r.ln = o.log_norm;
    }
    return r;
}

template <bool WL, typename ZT>
__device__ __forceinline__ double resolve_coord(const KleinArgs& a, int i, const ZT* Zp, size_t ldz,
                                                CoordStream& rs, double& lw, unsigned int& flags, double& tb) {
    const size_t iq = (size_t)i * kSzcStride;
    const Resolved r = resolve_decision(a.R, Zp, ldz, i, a.d, cst(a.cp)[i], cst(a.rii)[i],
                                        a.szc ? a.szc + iq : nullptr,
                                        a.szc ? cst(a.szc)[iq] : cst(a.sig)[i], rs.u((uint32_t)(a.d - 1 - i)),
                                        a.precision, a.linear_probs != 0, WL, a.etab,
                                        a.flags + kFlagWordResolved);
    if (!isfinite(r.mu)) {
        flags |= kFlagNonFinite;
        return 0.0;
    }
    lw += WL ? r.ln : ref_weight(r.z, r.mu, cst(a.ros)[i], cst(a.isr)[i], cst(a.lterm)[i]);
    if (WL) tb += fabs(r.ln);  // (a term at the reference-order mean: no bound)
    return r.z;
}


// Reference-order conditional mean of coordinate i of ONE sample (lane L of the
// calling wave), computed by the whole wave: lane k loads R_ij and z_j of
// j = j0 + k and forms the product (exactly the reference's rounded product), and
// the products are then added one at a time in ascending j (klein.py:191-195) --
// the serial part is 2 readlanes + 1 add per term instead of a latency-bound walk
// of one lane over R and its coefficients.  z_j: the int16 history (OZ; hL = the
// sample's base, exact for |z| <= 32639) or the coefficient store (zL = &Z[0][p]).
// All arguments wave-uniform; call from uniform control flow.
template <typename ZT>
__device__ __forceinline__ double mu_exact_wave(const double* __restrict__ R, const int16_t* __restrict__ hL,
                                                int64_t lanes, int shift, const ZT* __restrict__ zL,
                                                size_t ldz, int i, int d, double cp, double rii) {
    const int lane = threadIdx.x & 63;
    const double* __restrict__ Ri = R + (size_t)i * d;
    auto load = [&](int j0, double& r, double& z) {
        const int j = j0 + lane;
        r = 0.0;
        z = 0.0;
        if (j < d) {
            r = Ri[j];
            if (hL) {
                const int ih = j + shift;
                z = (double)((int)hL[(size_t)(ih >> 4) * lanes * 16 + (ih & 15)] - 128);
            } else {
                z = (double)zL[(size_t)j * ldz];
            }
        }
    };
    double cs = 0.0, r, z;
    load(i + 1, r, z);
    for (int j0 = i + 1; j0 < d; j0 += 64) {
        const double pr = r * z;  // this lane's term (unfused: -ffp-contract=off)
        if (j0 + 64 < d) load(j0 + 64, r, z);  // next chunk in flight
        const int m = min(64, d - j0);
        const long long bits = __double_as_longlong(pr);
        const int lo = (int)bits, hi = (int)(bits >> 32);
        for (int k = 0; k < m; ++k) {
            const long long b = ((long long)__builtin_amdgcn_readlane(hi, k) << 32) |
                                (unsigned int)__builtin_amdgcn_readlane(lo, k);
            cs = cs + __longlong_as_double(b);
        }
    }
    return (cp - cs) / rii;
}

// Verification of one 16-row sub-panel of klein_mfma_kernel (32-row panels), run by
// the whole wave when some lane has a decision the certificate did not cover
// (bits of fl: sub-panel step s; bit 16: the sub-panel's sum |z| exceeded the
// certificate's cap).  For each such lane L in turn, each uncovered decision is
// redone at the reference-order mean (mu_exact_wave, plain decision, same uniform):
// if every guess stands, only the skipped weight terms are added; otherwise (or
// with bit 16) the whole sub-panel is replayed in the reference's order from the
// weight and |z| sum of its start, rewriting L's coefficients and (OZ) history.
// The decisions of lane L are computed redundantly by every lane (uniform inputs).
// Returns the calling lane's weight, flags and nonzero bit (in registers: an output
// through a reference would keep the caller's copy in scratch memory, with a
// load-and-wait at every use); updates its |z| sum (z1l[lane]).
// A: the launch's arguments where the kernel received them (the kernarg segment,
// constant address space: scalar loads).  Taking the address of the by-value
// kernel argument instead makes the compiler copy the whole struct to scratch and
// read every field of it from there in the hot loop.
using KArgsPtr = const __attribute__((address_space(4))) KleinArgs*;
__device__ __forceinline__ KArgsPtr kernel_args() {
    return (KArgsPtr)__builtin_amdgcn_kernarg_segment_ptr();  // KleinArgs is argument 0: offset 0
}
struct VerifyOut {
    double lw;
    unsigned int flags;
    int nz;
    double tabs;  // (WL) sum |term| of the terms it added (reference-order means: no bound)
    double z2;    // sum z^2 of the calling lane's sub-panel after a replay of it, else -1
};
template <bool WL, bool OZ, typename ZT>
__device__ __noinline__ VerifyOut verify_subpanel(KArgsPtr A, ZT* __restrict__ Z, size_t ldz,
                                                  int64_t p0, int top, int rows, int fl, double lw,
                                                  uint32_t step, uint32_t chain, double* z1l,
                                                  const double* z1s, const double* lws, unsigned int flags) {
    int nz = 0;
    double tabs = 0.0, z2 = -1.0;
    const int lane = threadIdx.x & 63;
    const int d = A->d;
    // the sub-panel's coefficients / history were just stored by their own lanes and
    // are read here by the whole wave: write back and invalidate this CU's L1
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    uint64_t todo = __builtin_amdgcn_ballot_w64(fl != 0);
    while (todo) {
        const int L = __builtin_ctzll(todo);
        todo &= todo - 1;
        const int flL = __builtin_amdgcn_readlane(fl, L);
        const int64_t pL = p0 + L;
        const int16_t* hL = OZ ? A->h16 + (size_t)pL * 16 : nullptr;
        CoordStreamT<false> rs;
        rs.init(A->seed, (uint32_t)__builtin_amdgcn_readlane((int)step, L),
                (uint32_t)__builtin_amdgcn_readlane((int)chain, L));
        // plain (reference-mode) decision of lane L's coordinate i at mean mu
        auto decide = [&](int i, double mu, double& term, unsigned int& fb) -> double {
            const double* q = A->szc ? A->szc + (size_t)i * kSzcStride : nullptr;
            const double sg = q ? q[0] : A->sig[i];
            const double u = rs.u((uint32_t)(d - 1 - i));
            double zi = 0.0, ln = 0.0;
            if (!isfinite(mu)) {
                fb |= kFlagNonFinite;
                term = 0.0;
                return 0.0;
            }
            if (sg == 0.0) {
                zi = rint(mu);
            } else if (q) {
                zi = sample_z_coord(mu, u, (gdptr)q, A->precision, A->linear_probs != 0, WL, (gdptr)A->etab, ln,
                                    -1.0);
            } else {
                const SampleZOut o = sample_z(mu, sg, A->precision, A->linear_probs != 0, u, WL, A->etab);
                zi = (double)o.z;
                ln = o.log_norm;
            }
            term = WL ? ln : ref_weight(zi, mu, A->ros[i], A->isr[i], A->lterm[i]);
            return zi;
        };
        auto guess = [&](int i) -> double {  // lane L's stored coefficient
            if constexpr (OZ) {
                const int ih = i + A->h16_shift;
                return (double)((int)hL[(size_t)(ih >> 4) * A->h16_lanes * 16 + (ih & 15)] - 128);
            } else {
                return (double)Z[(size_t)i * ldz + pL];
            }
        };
        bool full = (flL >> 16) & 1;
        double dlw = 0.0, dtb = 0.0;
        unsigned int fb = 0;
        for (int s = 0; s < rows && !full; ++s) {
            if (!((flL >> s) & 1)) continue;
            const int i = top - 1 - s;
            const double mu = mu_exact_wave(A->R, hL, A->h16_lanes, A->h16_shift, Z + pL, ldz, i, d, A->cp[i], A->rii[i]);
            double term;
            const double zi = decide(i, mu, term, fb);
            if (zi != guess(i)) full = true;
            else dlw += term;
            dtb += fabs(term);
        }
        double z1n = 0.0, z2n = 0.0;
        int nzL = 0;
        if (full) {  // replay the sub-panel from its start
            dlw = 0.0;
            z1n = z1s[L];
            for (int s = 0; s < rows; ++s) {
                const int i = top - 1 - s;
                const double mu = mu_exact_wave(A->R, hL, A->h16_lanes, A->h16_shift, Z + pL, ldz, i, d, A->cp[i], A->rii[i]);
                double term;
                const double zi = decide(i, mu, term, fb);
                dlw += term;
                dtb += fabs(term);
                z1n += fabs(zi);
                z2n = fma(zi, zi, z2n);
                nzL |= zi != 0.0;
                if (lane == L) {
                    store_z(Z, (size_t)i * ldz + pL, zi, fb);
                    if constexpr (OZ) {
                        if (!(zi <= 32639.0 && zi >= -32767.0)) fb |= kFlagOverflow16;
                        const int ih = i + A->h16_shift;
                        A->h16[((size_t)(ih >> 4) * A->h16_lanes + pL) * 16 + (ih & 15)] =
                            (int16_t)(int)(fmin(fmax(zi, -32767.0), 32639.0) + 128.0);
                    }
                }
                // the wave's next reference-order sums read this coefficient
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
            }
        }
        if (lane == L) {
            flags |= fb;
            tabs += dtb;
            if (full) {
                lw = lws[L] + dlw;
                z1l[L] = z1n;
                z2 = z2n;
                nz |= nzL;
            } else {
                lw += dlw;
            }
        }
        if (lane == 0) atomicAdd(A->flags + kFlagWordResolved, 1u);
    }
    return VerifyOut{lw, flags, nz, tabs, z2};
}

// ------------------------------------------------------------ exact order
template <typename ZT, bool WL>
__global__ __launch_bounds__(256) void klein_exact_kernel(const KleinArgs a,
                                                          const double* __restrict__ R,
                                                          ZT* __restrict__ Z) {
    if (a.gate && *a.gate == 0u) return;  // whole grid: nothing to draw
    __shared__ double tab_lds[2 * (kErfTabLast + 1)];
    const lds_cdptr etab_s = stage_etab(tab_lds, a.etab);
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.n) return;
    uint32_t chain, step;
    lane_counter(a, p, chain, step);
    CoordStream rs;
    rs.init(a.seed, step, chain);
    const int d = a.d;
    const size_t ldz = (size_t)a.ldz;
    double lw = 0.0;
    unsigned int flags = 0;
    double eb = 0.0, tb = 0.0;
    for (int i = d - 1; i >= 0; --i) {
        const double* __restrict__ Ri = R + (size_t)i * d;
        double cs = 0.0;
        for (int j = i + 1; j < d; ++j) cs = cs + Ri[j] * (double)Z[(size_t)j * ldz + p];
        const double mu = (a.cp[i] - cs) / a.rii[i];
        const double zi = decide_coord<WL>(a, i, mu, rs, lw, flags, etab_s, -1.0, eb, tb);
        store_z(Z, (size_t)i * ldz + p, zi, flags);
    }
    if (a.LW) a.LW[p] = lw;
    if (a.LWE) a.LWE[p] = 0.0;  // the reference's order: exact
    if (flags) atomicOr(a.flags, flags);
}

// ------------------------------------------------------------ panel (fast)
// RP: far-field blocks, panel k (rows [p_hi-PB, p_hi), p_hi = d - k*PB) stores
//     for j in [p_hi, d): PB doubles RP[off_k + (j-p_hi)*PB + r] = R[p_hi-PB+r][j]
//     (0 for rows < 0); off_k = PB*PB*k*(k-1)/2.
// RC: near-field columns, RC[i*(PB-1) + m] = R[i-1-m][i] if row i-1-m is in
//     row i's panel, else 0.
template <typename ZT, int PB, bool WL>
__global__ __launch_bounds__(256) void klein_panel_kernel(const KleinArgs a,
                                                          const double* __restrict__ RP,
                                                          const double* __restrict__ RC,
                                                          ZT* __restrict__ Z) {
    if (a.gate && *a.gate == 0u) return;  // whole grid: nothing to draw
    __shared__ double tab_lds[2 * (kErfTabLast + 1)];
    const lds_cdptr etab_s = stage_etab(tab_lds, a.etab);
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.n) return;
    uint32_t chain, step;
    lane_counter(a, p, chain, step);
    CoordStream rs;
    rs.init(a.seed, step, chain);
    const int d = a.d;
    const size_t ldz = (size_t)a.ldz;
    double lw = 0.0;
    unsigned int flags = 0;
    const int npan = (d + PB - 1) / PB;
    double acc[PB];
    double z1 = 0.0;  // sum of |z_j| decided so far (certificate)
    double eb = 0.0, tb = 0.0;  // (WL) weight bound and sum |terms|
    for (int pk = 0; pk < npan; ++pk) {
        const int p_hi = d - pk * PB;
        const int rows = p_hi < PB ? p_hi : PB;
#pragma unroll
        for (int r = 0; r < PB; ++r) acc[r] = 0.0;
        const double* __restrict__ rp = RP + (size_t)PB * PB * ((size_t)pk * (pk - 1) / 2);
        int j = p_hi;
        for (; j + 1 < d; j += 2) {
            const double x0 = (double)Z[(size_t)j * ldz + p];
            const double x1 = (double)Z[(size_t)(j + 1) * ldz + p];
            const double* __restrict__ rj = rp + (size_t)(j - p_hi) * PB;
#pragma unroll
            for (int r = 0; r < PB; ++r) acc[r] = fma(rj[r], x0, acc[r]);
#pragma unroll
            for (int r = 0; r < PB; ++r) acc[r] = fma(rj[PB + r], x1, acc[r]);
        }
        if (j < d) {
            const double x0 = (double)Z[(size_t)j * ldz + p];
            const double* __restrict__ rj = rp + (size_t)(j - p_hi) * PB;
#pragma unroll
            for (int r = 0; r < PB; ++r) acc[r] = fma(rj[r], x0, acc[r]);
        }
        for (int s = 0; s < rows; ++s) {
            const int i = p_hi - 1 - s;
            const double mu = (cst(a.cp)[i] - acc[PB - 1]) * cst(a.irii)[i];
            double zi = decide_coord<WL>(a, i, mu, rs, lw, flags, etab_s,
                                         cert_dmu(cst(a.cert)[2 * i], cst(a.cert)[2 * i + 1], z1, mu), eb, tb);
            if (zi == kAmbiguous) zi = resolve_coord<WL>(a, i, Z + p, ldz, rs, lw, flags, tb);
            z1 += fabs(zi);
            store_z(Z, (size_t)i * ldz + p, zi, flags);
            const double x = zi;
            const cdptr rc = cst(RC) + (size_t)i * (PB - 1);
#pragma unroll
            for (int k = 0; k < PB - 1; ++k) acc[k] = fma(rc[PB - 2 - k], x, acc[k]);
#pragma unroll
            for (int k = PB - 1; k >= 1; --k) acc[k] = acc[k - 1];
            acc[0] = 0.0;
        }
    }
    if (a.LW) a.LW[p] = lw;
    if (WL) wl_bound_store(a, p, wl_bound_sum(eb, tb, d));
    if (flags) atomicOr(a.flags, flags);
}

// ------------------------------------------------------------ Babai nearest plane
// Deterministic twin of klein_panel_kernel: the same panel
// walk over R, with a per-target c' = Q^T t (coordinate-major CP[i][p]) and
// z_i = round-half-even((c'_i - sum_{j>i} R_ij z_j) / R_ii) -- the nearest-plane
// rule of src/lattices/base.py:105-135 in the QR frame (proj = <t, b*_i> /
// <b*_i, b*_i> with t updated by the decided coefficients), i.e. Klein's mean
// without the draw (klein.py:201-204).
template <typename ZT, int PB>
__global__ __launch_bounds__(256) void nearest_plane_kernel(int d, int64_t n,
                                                            const double* __restrict__ RP,
                                                            const double* __restrict__ RC,
                                                            const double* __restrict__ rii,
                                                            const double* __restrict__ CP, int64_t ldc,
                                                            ZT* __restrict__ Z, int64_t ldz_,
                                                            unsigned int* gflags) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const size_t ldz = (size_t)ldz_;
    unsigned int flags = 0;
    const int npan = (d + PB - 1) / PB;
    double acc[PB];
    for (int pk = 0; pk < npan; ++pk) {
        const int p_hi = d - pk * PB;
        const int rows = p_hi < PB ? p_hi : PB;
#pragma unroll
        for (int r = 0; r < PB; ++r) acc[r] = 0.0;
        const double* __restrict__ rp = RP + (size_t)PB * PB * ((size_t)pk * (pk - 1) / 2);
        int j = p_hi;
        for (; j + 1 < d; j += 2) {
            const double x0 = (double)Z[(size_t)j * ldz + p];
            const double x1 = (double)Z[(size_t)(j + 1) * ldz + p];
            const double* __restrict__ rj = rp + (size_t)(j - p_hi) * PB;
#pragma unroll
            for (int r = 0; r < PB; ++r) acc[r] = fma(rj[r], x0, acc[r]);
#pragma unroll
            for (int r = 0; r < PB; ++r) acc[r] = fma(rj[PB + r], x1, acc[r]);
        }
        if (j < d) {
            const double x0 = (double)Z[(size_t)j * ldz + p];
            const double* __restrict__ rj = rp + (size_t)(j - p_hi) * PB;
#pragma unroll
            for (int r = 0; r < PB; ++r) acc[r] = fma(rj[r], x0, acc[r]);
        }
        for (int s = 0; s < rows; ++s) {
            const int i = p_hi - 1 - s;
            const double mu = (CP[(size_t)i * ldc + p] - acc[PB - 1]) / cst(rii)[i];
            double zi = 0.0;
            if (isfinite(mu))
                zi = rint(mu);
            else
                flags |= kFlagNonFinite;
            store_z(Z, (size_t)i * ldz + p, zi, flags);
            const cdptr rc = cst(RC) + (size_t)i * (PB - 1);
#pragma unroll
            for (int k = 0; k < PB - 1; ++k) acc[k] = fma(rc[PB - 2 - k], zi, acc[k]);
#pragma unroll
            for (int k = PB - 1; k >= 1; --k) acc[k] = acc[k - 1];
            acc[0] = 0.0;
        }
    }
    if (flags) atomicOr(gflags, flags);
}

// Babai rounding (src/lattices/simple.py:112-128, src/samplers/utils.py:575-577):
// z = round-half-even(w), w = B^{-1} t given coordinate-major.
template <typename ZT>
__global__ __launch_bounds__(256) void round_kernel(const double* __restrict__ W, int64_t ldw, int d,
                                                    int64_t n, ZT* __restrict__ Z, int64_t ldz,
                                                    unsigned int* gflags) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    if (p >= n) return;
    unsigned int flags = 0;
    const double w = W[(size_t)i * ldw + p];
    double zi = 0.0;
    if (isfinite(w))
        zi = rint(w);
    else
        flags |= kFlagNonFinite;
    store_z(Z, (size_t)i * ldz + p, zi, flags);
    if (flags) atomicOr(gflags, flags);
}

// ------------------------------------------------------------ panel, MFMA far field
// Same sampler and panel layout as klein_panel_kernel (PB = 16 or 32 rows), but
// the far-field product of a panel -- F[PB rows][64 chains] = R_panel[PB x K] *
// X[K x 64 chains], K = d - p_hi -- runs on the matrix cores of the wave:
// v_mfma_f64_16x16x4_f64, one 16-row tile t per MFMA, A = R tile (lane l:
// R[p_lo + 16t + (l&15)][j0 + (l>>4)], coalesced 512 B) and B = coefficients
// (lane l loads 4 consecutive chains of row j0 + (l>>4) in one load; MFMA g takes
// chain 4n+g, n = l&15), so one coefficient load feeds PB/16 * 4 MFMAs.
// D (lane l: rows (l>>4)+4*reg, chain 4*(l&15)+g) is transposed to one chain per
// lane through a per-wave 8 KB LDS tile; the near field and SampleZ then run on
// the VALU exactly as in klein_panel_kernel.  Requires n % 64 == 0, ldz % 4 == 0.
// Coefficients written by other lanes are read back with L1-bypassing (nt) loads
// after a wavefront release (s_waitcnt vmcnt(0)).
typedef int v4i32_t __attribute__((ext_vector_type(4)));
typedef double d4_t __attribute__((ext_vector_type(4)));

// Four consecutive coefficients of one coordinate row (one MFMA B fragment
// column group), loaded with ordinary (temporal) loads -- measured ~1% faster
// than non-temporal ones on MI355X; raw storage per type, converted to fp64
// when the MFMA consumes them (64-bit values are converted exactly).
template <typename ZT>
struct ZQuad;
template <>
struct ZQuad<int16_t> {
    unsigned long long w;
    __device__ __forceinline__ void load(const int16_t* p) {
        w = *(const unsigned long long*)p;
    }
    __device__ __forceinline__ double get(int g) const { return (double)(short)(w >> (16 * g)); }
};
template <>
struct ZQuad<int32_t> {
    v4i32_t v;
    __device__ __forceinline__ void load(const int32_t* p) {
        v = *(const v4i32_t*)p;
    }
    __device__ __forceinline__ double get(int g) const { return (double)v[g]; }
};
template <>
struct ZQuad<int64_t> {
    long long v[4];
    __device__ __forceinline__ void load(const int64_t* p) {
#pragma unroll
        for (int g = 0; g < 4; ++g) v[g] = ((const long long*)p)[g];
    }
    __device__ __forceinline__ double get(int g) const { return (double)v[g]; }
};

// ---------------------------------------------------- int8-digit far field
// F_i = sum_{j >= p_hi} R_ij x_j for the 32 rows of panel pk and the wave's 64
// samples, exactly enough to stand in for fp64: rows scaled by 2^E_i and split
// into kOzDigits = 6 balanced base-256 digits r_a (|R 2^-E| < 1/4, rounded to
// 2^(E-48); host: lgs_set_basis, whose certificate bound covers the rounding); coefficients x in [-32767, 32639] held in the int16
// history as y = x + 128, so x = 256 x1 + x0 with x1 = the high byte of y and
// x0 = low byte ^ 0x80 (both signed): a digit plane is two byte permutes of the
// raw int16 pairs, and x = 0 gives two zero planes.  Class c = a - b of r_a x_b
// (weight 256^-c) is summed exactly in int32 on v_mfma_i32_16x16x64_i8
// (|sum| <= 2 K 2^14 < 2^31 for d <= 32768); then F_i = 2^E_i sum_c 256^-c C_c
// (classes c = 0 .. kOzDigits).
// Chunks whose two 32-row panels are zero in every sample of the block (bits of
// nzm, set by the near field) contribute nothing and are skipped: no history
// read, no slab, no MFMA.
// Four passes (16 samples each) keep 2 row tiles x 7 classes = 56 accumulator
// VGPRs.  Row tile 1 (the upper sub-panel) goes to acc through the LDS tile;
// tile 0 is parked in the per-wave scratch f0 and moved into the LDS tile once
// the upper rows are loaded (the LDS tile is free during the upper sub-panel).
#ifdef LGS_DIAG_FAR  // diagnostic builds only: per-wave shader-clock phases of the far field's chunk loop
__device__ unsigned long long lgs_diag_far[8];  // [0] history wait [1] slab store [2] MFMA issue [3] barrier
                                                // [4] prologue [5] epilogue [6] chunk visits [7] calls
#define LGS_DF_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#else
#define LGS_DF_T(v)
#endif
#ifndef LGS_OZ_NG  // 16-sample groups per far-field pass (1 or 2)
#define LGS_OZ_NG 2
#endif

__device__ __forceinline__ void oz_far_field(const KleinArgs& a, int pk, int p_hi, int64_t p0, int lane,
                                             lds_cdptr rec, double* F, int LDF, double (&acc)[16],
                                             int8_t* ash, const uint32_t* nzm, bool coarse = false) {
    const int d = a.d;
    const int K = d - p_hi, nch = (K + 63) / 64;
    // chunk ch covers panels pk-1-2ch and pk-2-2ch (panel q: rows d-32(q+1) .. d-32q-1)
    auto live = [&](int ch) -> bool {
        const int q0 = pk - 1 - 2 * ch, q1 = q0 - 1;
        uint32_t b = nzm[q0 >> 5] >> (q0 & 31);
        if (q1 >= 0) b |= nzm[q1 >> 5] >> (q1 & 31);
        return (__builtin_amdgcn_readfirstlane(b) & 1u) != 0;
    };
    auto next_live = [&](int ch) {
        while (ch < nch && !live(ch)) ++ch;
        return ch;
    };
    const int h = lane >> 4, n = lane & 15, tid = threadIdx.x;
    // block-shared R-digit slab of one 64-column chunk (both row tiles): 896 x 16 B,
    // double-buffered in LDS; thread tid stages pieces tid + 256 m (m < 4, < 896)
    constexpr int SLAB = 2 * kOzDigits * 64;
    const v4i32_t* __restrict__ rsrc =
        (const v4i32_t*)(a.rd + ((const __attribute__((address_space(4))) int64_t*)a.rd_off)[pk]);
    v4i32_t* ash4 = (v4i32_t*)ash;
    const size_t blk0 = (size_t)((p_hi + a.h16_shift) >> 4) + h;
    const size_t hstep = (size_t)4 * a.h16_lanes * 16;  // 4 history blocks = one 64-column chunk
    double t0v[4][4];  // lower row tile, D layout, until the LDS tile is free
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) t0v[g][reg] = 0.0;
#ifdef LGS_XP_ALIAS
    // the upper row tile too: F shares its LDS with the slab, which later passes still use
    double t1v[4][4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) t1v[g][reg] = 0.0;
#endif
    // piece e of the slab is fragment e / 64 = (tile, digit) = ((e / 64) / kOzDigits, (e / 64) % kOzDigits);
    // a coarse panel's MFMAs read only the kOzCoarse most significant digits: the other
    // pieces are neither loaded nor staged (LGS_OZ_COARSE_FULL_SLAB: staged, round 5)
    auto piece_used = [&](int e) {
#ifndef LGS_OZ_COARSE_FULL_SLAB
        return e < SLAB && (!coarse || (e >> 6) % kOzDigits < kOzCoarse);
#else
        return e < SLAB;
#endif
    };
    auto slab_load = [&](int ch, v4i32_t (&pf)[4]) {
#ifdef LGS_DIAG_FAR_NOSLAB
        ch = 0;
#endif
        const v4i32_t* src = rsrc + (size_t)ch * SLAB;
#pragma unroll
        for (int m = 0; m < 4; ++m)
            if (piece_used(tid + 256 * m)) pf[m] = src[tid + 256 * m];
    };
    auto slab_store = [&](int buf, const v4i32_t (&pf)[4]) {
#ifdef LGS_DIAG_FAR_NOSLAB  // diagnostic builds only (NOT bit-exact): no R-digit slab traffic (stale LDS)
        asm volatile("" ::"v"(pf[0]));
        return;
#endif
#pragma unroll
        for (int m = 0; m < 4; ++m)
            if (piece_used(tid + 256 * m)) ash4[buf * SLAB + tid + 256 * m] = pf[m];
    };
    // 4/NG passes of NG 16-sample groups: each A fragment read from LDS feeds 2 NG MFMAs
    constexpr int NG = LGS_OZ_NG;
#ifdef LGS_DIAG_FAR
    uint64_t df[8] = {};
    LGS_DF_T(tf_begin);
#endif
#ifdef LGS_OZ_PIPE_PASSES
    // (round 6, measured and kept out: C3 7.90-8.07 vs 7.86-7.91 ms, C4 11.90-11.94 vs
    // 11.79-11.81 ms per 2^20, profiles/r06g_kb.log) The passes as one pipelined sequence of (pass, live chunk) items:
    // the loads of a pass's first chunk (history and R-digit slab) are issued during the
    // previous pass's last chunk, as within a pass, instead of in a prologue of their
    // own whose latency nothing hid; each pass's classes are recombined behind the
    // barrier of its last chunk, while the next item's loads are in flight.
    {
        constexpr int NP = 4 / NG;
        constexpr int NC = kOzDigits + 1;  // digit classes
        v4i32_t cc[NG][2][NC];  // [group][row tile][class]
        auto cc_zero = [&]() {
#pragma unroll
            for (int q = 0; q < NG; ++q)
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int c = 0; c < NC; ++c) cc[q][t][c] = (v4i32_t){0, 0, 0, 0};
        };
        cc_zero();
        v4i32_t pf[4];
        v4u_t w[NG][2];
        auto hist_load = [&](int gp, int ch) {
            const int16_t* __restrict__ hb0 = a.h16 + (blk0 * a.h16_lanes + p0 + 16 * NG * gp + n) * 16;
            const v4u_t* h0 = (const v4u_t*)(hb0 + (size_t)ch * hstep);
            w[0][0] = *(h0);
            w[0][1] = *(h0 + 1);
            if constexpr (NG == 2) {
                const v4u_t* h1 = (const v4u_t*)(hb0 + 16 * 16 + (size_t)ch * hstep);  // group NG gp + 1
                w[NG - 1][0] = *(h1);
                w[NG - 1][1] = *(h1 + 1);
            }
        };
        // classes -> fp64; D layout: rows 4h + reg of the tile, sample 16g + n
        auto epilogue = [&](int gp) {
#pragma unroll
            for (int q = 0; q < NG; ++q)
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int reg = 0; reg < 4; ++reg) {
                        const int g = NG * gp + q;
                        const int row = 16 * t + 4 * h + reg;  // panel row = record index
                        double sv = (double)cc[q][t][NC - 1][reg];
#pragma unroll
                        for (int c = NC - 2; c >= 0; --c) sv = fma(sv, 0.00390625, (double)cc[q][t][c][reg]);
                        const double fv = sv * rec[row * kRecStride + kRecScale];
                        if (t == 1) {
#ifdef LGS_XP_ALIAS
#pragma unroll
                            for (int gg = 0; gg < 4; ++gg) t1v[gg][reg] = g == gg ? fv : t1v[gg][reg];
#else
                            F[(4 * h + reg) * LDF + 16 * g + n] = fv;
#endif
                        } else {
#pragma unroll
                            for (int gg = 0; gg < 4; ++gg) t0v[gg][reg] = g == gg ? fv : t0v[gg][reg];
                        }
                    }
            cc_zero();
        };
        // (no barrier needed first: the panel's record-staging barrier also publishes nzm)
        const int first = next_live(0);
        if (first >= nch) {
#pragma unroll 1
            for (int gp = 0; gp < NP; ++gp) epilogue(gp);
        } else {
            // the item after (g, c): the next live chunk of pass g, else pass g + 1's first
            auto advance = [&](int& g, int& c) {
                c = next_live(c + 1);
                if (c >= nch) {
                    c = first;
                    ++g;
                }
            };
            int cgp = 0, cur = first;
            int ngp = 0, nxt = first;
            advance(ngp, nxt);
            slab_load(cur, pf);
            slab_store(0, pf);
            if (ngp < NP) slab_load(nxt, pf);
            hist_load(cgp, cur);
            __syncthreads();
#pragma unroll 1
            for (int it = 0; cgp < NP; ++it) {
                v4i32_t xh[NG], xl[NG];  // history of chunk cur -> digit planes, per group
#pragma unroll
                for (int q = 0; q < NG; ++q) {
                    const v4u_t w0 = w[q][0], w1 = w[q][1];
                    xh[q][0] = (int)__builtin_amdgcn_perm(w0[1], w0[0], 0x07050301u);
                    xh[q][1] = (int)__builtin_amdgcn_perm(w0[3], w0[2], 0x07050301u);
                    xh[q][2] = (int)__builtin_amdgcn_perm(w1[1], w1[0], 0x07050301u);
                    xh[q][3] = (int)__builtin_amdgcn_perm(w1[3], w1[2], 0x07050301u);
                    xl[q][0] = (int)(__builtin_amdgcn_perm(w0[1], w0[0], 0x06040200u) ^ 0x80808080u);
                    xl[q][1] = (int)(__builtin_amdgcn_perm(w0[3], w0[2], 0x06040200u) ^ 0x80808080u);
                    xl[q][2] = (int)(__builtin_amdgcn_perm(w1[1], w1[0], 0x06040200u) ^ 0x80808080u);
                    xl[q][3] = (int)(__builtin_amdgcn_perm(w1[3], w1[2], 0x06040200u) ^ 0x80808080u);
                }
                int ngp2 = ngp, nxt2 = nxt;
                if (ngp < NP) {  // the next item's history; its slab -> LDS, fetch the one after
                    advance(ngp2, nxt2);
                    hist_load(ngp, nxt);
                    slab_store((it + 1) & 1, pf);
                    if (ngp2 < NP) slab_load(nxt2, pf);
                }
                const v4i32_t* sl = ash4 + (it & 1) * SLAB + lane;
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int dg = 0; dg < kOzDigits; ++dg) {
                        // coarse (wave-uniform): only the kOzCoarse most significant digits
                        if (dg >= kOzCoarse && coarse) continue;
                        const v4i32_t av = sl[(t * kOzDigits + dg) * 64];
                        // digit a = dg + 1: class a - 1 with the high x digit, class a with the low
#pragma unroll
                        for (int q = 0; q < NG; ++q) {
                            cc[q][t][dg] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, xh[q], cc[q][t][dg], 0, 0, 0);
                            cc[q][t][dg + 1] =
                                __builtin_amdgcn_mfma_i32_16x16x64_i8(av, xl[q], cc[q][t][dg + 1], 0, 0, 0);
                        }
                    }
                __syncthreads();  // next slab complete; this one's reads done before it is reused
                if (ngp != cgp) epilogue(cgp);  // (the pass's last chunk)
                cgp = ngp;
                cur = nxt;
                ngp = ngp2;
                nxt = nxt2;
            }
        }
    }
#else
#pragma unroll 1
    for (int gp = 0; gp < 4 / NG; ++gp) {
        constexpr int NC = kOzDigits + 1;  // digit classes
        v4i32_t cc[NG][2][NC];  // [group][row tile][class]
#pragma unroll
        for (int q = 0; q < NG; ++q)
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int c = 0; c < NC; ++c) cc[q][t][c] = (v4i32_t){0, 0, 0, 0};
        const int16_t* __restrict__ hb0 = a.h16 + (blk0 * a.h16_lanes + p0 + 16 * NG * gp + n) * 16;
        const int16_t* __restrict__ hb1 = hb0 + 16 * 16;  // group NG gp + 1: 16 lanes further
        v4i32_t pf[4];
        v4u_t w[NG][2];
        auto hist_load = [&](int ch) {
#ifdef LGS_DIAG_HIST_FIXED  // diagnostic builds only (NOT bit-exact): every chunk reads chunk 0's history
            ch = 0;
#endif
            const v4u_t* h0 = (const v4u_t*)(hb0 + (size_t)ch * hstep);
            const v4u_t* h1 = (const v4u_t*)(hb1 + (size_t)ch * hstep);
            w[0][0] = *(h0);
            w[0][1] = *(h0 + 1);
            if constexpr (NG == 2) {
                w[NG - 1][0] = *(h1);
                w[NG - 1][1] = *(h1 + 1);
            } else {
                (void)h1;
            }
        };
#ifdef LGS_OZ_PASS_BARRIER
        __syncthreads();  // previous pass done with both buffers
#endif
        // (no barrier needed here: the previous pass's chunk loop ended with one after
        // its last slab reads, and pass 0 follows the panel's record-staging barrier,
        // which also publishes nzm)
        int cur = next_live(0);
        int nxt = cur < nch ? next_live(cur + 1) : nch;
#ifdef LGS_DIAG_FAR
        LGS_DF_T(tp0);
#endif
        if (cur < nch) {
            slab_load(cur, pf);
            slab_store(0, pf);
            if (nxt < nch) slab_load(nxt, pf);
            hist_load(cur);
        }
        __syncthreads();
#ifdef LGS_DIAG_FAR
        {
            LGS_DF_T(tp1);
            df[4] += tp1 - tp0;
        }
#endif
#pragma unroll 1
        for (int it = 0; cur < nch; ++it) {
#ifdef LGS_DIAG_FAR
            LGS_DF_T(tc0);
#endif
            v4i32_t xh[NG], xl[NG];  // history of chunk ch -> digit planes, per group
#pragma unroll
            for (int q = 0; q < NG; ++q) {
                const v4u_t w0 = w[q][0], w1 = w[q][1];
                xh[q][0] = (int)__builtin_amdgcn_perm(w0[1], w0[0], 0x07050301u);
                xh[q][1] = (int)__builtin_amdgcn_perm(w0[3], w0[2], 0x07050301u);
                xh[q][2] = (int)__builtin_amdgcn_perm(w1[1], w1[0], 0x07050301u);
                xh[q][3] = (int)__builtin_amdgcn_perm(w1[3], w1[2], 0x07050301u);
                xl[q][0] = (int)(__builtin_amdgcn_perm(w0[1], w0[0], 0x06040200u) ^ 0x80808080u);
                xl[q][1] = (int)(__builtin_amdgcn_perm(w0[3], w0[2], 0x06040200u) ^ 0x80808080u);
                xl[q][2] = (int)(__builtin_amdgcn_perm(w1[1], w1[0], 0x06040200u) ^ 0x80808080u);
                xl[q][3] = (int)(__builtin_amdgcn_perm(w1[3], w1[2], 0x06040200u) ^ 0x80808080u);
            }
#ifdef LGS_DIAG_FAR
            asm volatile("" ::"v"(xh[NG - 1]), "v"(xl[NG - 1]));
            LGS_DF_T(tc1);
#endif
            const int nxt2 = nxt < nch ? next_live(nxt + 1) : nch;
            if (nxt < nch) {  // history of the next live chunk; its slab -> LDS, fetch the one after
                hist_load(nxt);
                slab_store((it + 1) & 1, pf);
                if (nxt2 < nch) slab_load(nxt2, pf);
            }
#ifdef LGS_DIAG_FAR
            LGS_DF_T(tc2);
#endif
            const v4i32_t* sl = ash4 + (it & 1) * SLAB + lane;
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int dg = 0; dg < kOzDigits; ++dg) {
                    // coarse (wave-uniform): only the kOzCoarse most significant digits
                    if (dg >= kOzCoarse && coarse) continue;
                    const v4i32_t av = sl[(t * kOzDigits + dg) * 64];
                    // digit a = dg + 1: class a - 1 with the high x digit, class a with the low
#ifdef LGS_DIAG_FAR_NOMFMA  // diagnostic builds only (NOT bit-exact): the far field's loads and barriers alone
                    asm volatile("" ::"v"(av), "v"(xh[NG - 1]), "v"(xl[NG - 1]));
                    continue;
#endif
#pragma unroll
                    for (int q = 0; q < NG; ++q) {
                        cc[q][t][dg] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, xh[q], cc[q][t][dg], 0, 0, 0);
                        cc[q][t][dg + 1] =
                            __builtin_amdgcn_mfma_i32_16x16x64_i8(av, xl[q], cc[q][t][dg + 1], 0, 0, 0);
                    }
                }
#ifdef LGS_DIAG_FAR
            LGS_DF_T(tc3);
#endif
            __syncthreads();  // next slab complete; this one's reads done before it is reused
#ifdef LGS_DIAG_FAR
            {
                LGS_DF_T(tc4);
                df[0] += tc1 - tc0;
                df[1] += tc2 - tc1;
                df[2] += tc3 - tc2;
                df[3] += tc4 - tc3;
                df[6] += 1;
            }
#endif
            cur = nxt;
            nxt = nxt2;
        }
        // classes -> fp64; D layout: rows 4h + reg of the tile, sample 16g + n
#pragma unroll
        for (int q = 0; q < NG; ++q)
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int reg = 0; reg < 4; ++reg) {
                    const int g = NG * gp + q;
                    const int row = 16 * t + 4 * h + reg;  // panel row = record index
                    double sv = (double)cc[q][t][NC - 1][reg];
#pragma unroll
                    for (int c = NC - 2; c >= 0; --c) sv = fma(sv, 0.00390625, (double)cc[q][t][c][reg]);
                    const double fv = sv * rec[row * kRecStride + kRecScale];
                    if (t == 1) {
#ifdef LGS_XP_ALIAS
#pragma unroll
                        for (int gg = 0; gg < 4; ++gg) t1v[gg][reg] = g == gg ? fv : t1v[gg][reg];
#else
                        F[(4 * h + reg) * LDF + 16 * g + n] = fv;
#endif
                    } else {
#pragma unroll
                        for (int gg = 0; gg < 4; ++gg) t0v[gg][reg] = g == gg ? fv : t0v[gg][reg];
                    }
                }
    }
#endif
#ifdef LGS_XP_ALIAS
    // every pass's chunk loop ended with a block barrier after its last slab reads (and
    // a block without live chunks never touched the slab): F is free for every wave
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) F[(4 * h + reg) * LDF + 16 * g + n] = t1v[g][reg];
#endif
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = F[r * LDF + lane];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) F[(4 * h + reg) * LDF + 16 * g + n] = t0v[g][reg];
#ifdef LGS_DIAG_FAR
    {
        LGS_DF_T(tf_end);
        df[7] += 1;
        // epilogue = the whole call minus prologues and loops
        df[5] += (tf_end - tf_begin) - df[0] - df[1] - df[2] - df[3] - df[4];
        if ((threadIdx.x & 63) == 0)
            for (int k = 0; k < 8; ++k) atomicAdd(&lgs_diag_far[k], (unsigned long long)df[k]);
    }
#endif
}

#ifndef LGS_MFMA_LB32
#define LGS_MFMA_LB32 3
#endif
#ifndef LGS_OZ_LB  // waves per SIMD the int8-digit far-field kernel is compiled for
#define LGS_OZ_LB 2
#endif
// Diagnostic builds (-DLGS_DIAG_CYCLES): per-wave shader-clock accounting of the
// 32-row-panel kernel, summed over waves into lgs_diag_cycles (lane 0 adds):
// [0] record staging + barriers, [1] far field, [2] near field, [3 + kind] the
// SampleZ decision (with its Philox draw) per SampleZ kind, [8 + kind] decisions
// per kind, [13] whole kernel.
#ifdef LGS_DIAG_CYCLES
__device__ unsigned long long lgs_diag_cycles[16];
#define LGS_DC_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define LGS_DC_ADD(k, x) dc[k] += (x)
#else
#define LGS_DC_T(v)
#define LGS_DC_ADD(k, x)
#endif
// OZ (32-row panels only): far field as an exact int8-digit product on
// v_mfma_i32_16x16x64_i8 instead of fp64 MFMA (see oz_far_field).
template <typename ZT, int PB, bool WL, bool OZ = false, bool LIBM = false>
__global__ __launch_bounds__(256, PB == 32 ? (OZ ? LGS_OZ_LB : LGS_MFMA_LB32) : 3) void klein_mfma_kernel(const KleinArgs a,
                                                            const double* __restrict__ RP,
                                                            const double* __restrict__ RC,
                                                            ZT* __restrict__ Z) {
    if (a.gate && *a.gate == 0u) return;  // whole grid: nothing to draw
    constexpr int NT = PB / 16, LDF = 65;  // LDS tile pitch (doubles): conflict-free row reads
#ifdef LGS_XP_ALIAS  // (experiment: the far-field tiles share the R-digit slab's LDS)
    __shared__ __attribute__((aligned(16))) double Fl_raw[4 * 16 * LDF];
    double (*Fl)[16 * LDF] = (double (*)[16 * LDF])Fl_raw;
#else
    __shared__ double Fl[4][16 * LDF];
#endif
    // OZ: the erf table stays in global memory (L1-resident lookups measured as fast
    // as LDS) to leave LDS for the block-shared R-digit slab of the far field
    __shared__ double tab_lds[OZ ? 2 : 2 * (kErfTabLast + 1)];
#ifdef LGS_XP_ALIAS
    int8_t* ash = (int8_t*)Fl_raw;
#else
    __shared__ __attribute__((aligned(16))) int8_t ash[OZ ? 2 * 2 * kOzDigits * 1024 : 16];  // 2 x 14 KB
#endif
#ifdef LGS_COEF_ON  // Taylor-coefficient table: measured 2% slower (load latency)
    using ETP = std::conditional_t<OZ, CoefTab, lds_cdptr>;
    ETP etab_s;
    if constexpr (OZ)
        etab_s = CoefTab{a.etab2};
    else
        etab_s = stage_etab(tab_lds, a.etab);
#else
    using ETP = std::conditional_t<OZ, gdptr, lds_cdptr>;
    ETP etab_s;
    if constexpr (OZ)
        etab_s = (gdptr)a.etab;
    else
        etab_s = stage_etab(tab_lds, a.etab);
#endif
    // 32-row panels: the panel's per-coordinate records, staged block-wide
    __shared__ __attribute__((aligned(16))) double rec_lds[PB == 32 ? 32 * kRecStride : 2];
    // OZ: bit q set when panel q has a nonzero coefficient in some sample of the block
    __shared__ uint32_t nzm[OZ ? kOzMaxD / 32 / 32 : 1];
    if constexpr (OZ)
        for (int e = threadIdx.x; e < kOzMaxD / 32 / 32; e += 256) nzm[e] = 0u;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#ifdef LGS_DIAG_CYCLES
    uint64_t dc[16] = {};
#endif
    LGS_DC_T(t_kernel0);
    const int64_t p0 = ((int64_t)blockIdx.x * 4 + wave) * 64;
    const bool active = p0 < a.n;  // whole waves only (n % 64 == 0)
    if (!active && PB != 32) return;  // (32-row panels: idle waves still stage records)
    const int64_t p = p0 + lane;
    uint32_t chain, step;
    lane_counter(a, p, chain, step);
    CoordStream rs;
    rs.init(a.seed, step, chain);
    const int d = a.d;
    const size_t ldz = (size_t)a.ldz;
    double lw = 0.0;
    unsigned int flags = 0;
    const int npan = (d + PB - 1) / PB;
    double* F = Fl[wave];
    const int kq = lane >> 4, nq = lane & 15;
    constexpr int NACC = PB == 32 ? 16 : PB;  // running sums live across SampleZ calls
    double acc[NACC];
    double z1 = 0.0;  // sum of |z_j| decided so far (certificate; 16-row panels)
    double eb = 0.0, tb = 0.0;  // (WL) weight bound and sum |terms| (wl_bound_*)
    // 32-row panels, per lane in LDS (a live register pair across the near field
    // measured 0.7 ms slower per 2^20 samples): [0] the running sum of |z_j|, [1] it
    // and [2] the weight at the start of the current sub-panel (for a replay)
    __shared__ double cert_lds[3][PB == 32 ? 256 : 1];
    // bit s: decision s of the current sub-panel not covered by the certificate (in
    // LDS, written only when set: a live mask register costs ~13 scratch ops per
    // coordinate at this kernel's register pressure)
#ifdef LGS_NEAR_UNROLLED
    __shared__ int cert_fl[PB == 32 ? 256 : 1];
#endif
    // q-panel skip (reference mode, a.qz2): per lane sum z_j^2 over the coordinates
    // outside speculative sub-panels (+inf once a speculative coordinate is nonzero),
    // and the block's vote for skipping the current panel
    __shared__ double qzs[PB == 32 ? 256 : 1];
#ifdef LGS_QSKIP_STAGED
    __shared__ int qskip_blk[2];  // (by panel parity: a wave may start the next panel before another
                                  // has read this panel's vote when there is no block barrier between)
#else
    // each wave's vote, by panel parity (a wave reaches panel pk + 2 only after every wave
    // has passed panel pk + 1's barrier, i.e. read panel pk's votes)
    __shared__ int qvote[2][4];
#endif
    if constexpr (PB == 32) {
        cert_lds[0][threadIdx.x] = 0.0;
#ifdef LGS_NEAR_UNROLLED
        cert_fl[threadIdx.x] = 0;
#endif
        qzs[threadIdx.x] = 0.0;
    }
    for (int pk = 0; pk < npan; ++pk) {
        const int p_hi = d - pk * PB;
        const int rows = p_hi < PB ? p_hi : PB;
        LGS_DC_T(t_panel0);
        if constexpr (PB == 32) {
            // q-panel skip (reference mode): a panel of 32 small-kind rows whose means the
            // host bounds by Cauchy-Schwarz, |mu_i| <= (|c'_i| + (1 + g) G_i ||z_W||) / R_ii
            // (G_i = ||R[i, W]||, W = the coordinates outside speculative sub-panels, valid
            // while every speculative z so far is 0), is decided z = 0 in every row with
            // certainty when ||z_W||^2 <= qz2[pk] (the one-dominant-point test passes for
            // every |mu| below the bound, lgs_set_basis): no far field, no means.  The
            // weight term of such a row is taken at mu = 0: ref_weight(0, 0) = lterm
            // exactly, against lterm + 0.5 mu^2 (isr^2 - ros^2) ~ lterm + 1e-15 at the
            // blocked mean (isr and ros are R_ii / sigma in two roundings).  Block-wide
            // (the far field stages the R-digit slab with block barriers).
            bool qtry = false;
#if !defined(LGS_NEAR_UNROLLED) && !defined(LGS_NO_QSKIP_CODE)  // (that variant does not track ||z_W||)
            if constexpr (OZ && !WL)
                qtry = a.qz2 != nullptr && p_hi >= 32 && ((const __attribute__((address_space(4))) double*)a.qz2)[pk] >= 0.0;
#endif
            const int r0 = p_hi - 32;
#ifdef LGS_QSKIP_STAGED  // (round 5: the panel's records staged before the vote is read)
            // records of coordinates r0 .. r0+31 (r0 = p_hi - 32; negative ones skipped)
            if (qtry && threadIdx.x == 0) qskip_blk[pk & 1] = 1;  // (read last at panel pk - 2: done)
            __syncthreads();
            if (qtry) {
                const double q2 = ((const __attribute__((address_space(4))) double*)a.qz2)[pk];
                if (__builtin_amdgcn_ballot_w64(active && !(qzs[threadIdx.x] <= q2)) != 0 && lane == 0)
                    qskip_blk[pk & 1] = 0;
            }
            bool skip = false;
            {
                const double2* __restrict__ src = (const double2*)a.crec;
                double2* dst = (double2*)rec_lds;
                for (int e = threadIdx.x; e < 32 * kRecStride / 2; e += 256)
                    if (r0 * (kRecStride / 2) + e >= 0) dst[e] = src[(int64_t)r0 * (kRecStride / 2) + e];
                __syncthreads();
                skip = qtry && __builtin_amdgcn_readfirstlane(qskip_blk[pk & 1]) != 0;
            }
#else
            // (round 6) each wave votes before the barrier that ends the previous panel; a
            // panel the block skips stages no records (the weight terms are read from the
            // record array in memory) and needs no second barrier
            if (qtry) {
                const double q2 = ((const __attribute__((address_space(4))) double*)a.qz2)[pk];
                const bool ok = __builtin_amdgcn_ballot_w64(active && !(qzs[threadIdx.x] <= q2)) == 0;
                if (lane == 0) qvote[pk & 1][wave] = ok ? 1 : 0;
            }
            __syncthreads();  // the previous panel's record reads done; the votes visible
            const bool skip = qtry && __builtin_amdgcn_readfirstlane(qvote[pk & 1][0] & qvote[pk & 1][1] &
                                                                     qvote[pk & 1][2] & qvote[pk & 1][3]) != 0;
            if (!skip) {
                // records of coordinates r0 .. r0+31 (r0 = p_hi - 32; negative ones skipped)
                const double2* __restrict__ src = (const double2*)a.crec;
                double2* dst = (double2*)rec_lds;
                for (int e = threadIdx.x; e < 32 * kRecStride / 2; e += 256)
                    if (r0 * (kRecStride / 2) + e >= 0) dst[e] = src[(int64_t)r0 * (kRecStride / 2) + e];
                __syncthreads();
            }
#endif
            if (!active) continue;
            if (skip) {
                if (lane == 0) atomicAdd(a.flags + kFlagWordQSkip, 1u);
                // the 32 weight terms from the contiguous per-coordinate array (one batch of
                // scalar loads), added in the sequential order
                const cdptr lt = uniformize(cst(a.lterm) + r0);
                double ltv[32];
#pragma unroll
                for (int s = 0; s < 32; ++s) ltv[s] = lt[31 - s];
#pragma unroll
                for (int s = 0; s < 32; ++s) {
                    Z[(size_t)(p_hi - 1 - s) * ldz + p] = (ZT)0;
                    lw += ltv[s];
                }
                v4u_t* hp4 = (v4u_t*)(a.h16 + ((size_t)((p_hi - 32 + a.h16_shift) >> 4) * a.h16_lanes + p) * 16);
                const v4u_t h128 = (v4u_t){0x00800080u, 0x00800080u, 0x00800080u, 0x00800080u};
                hp4[0] = h128;
                hp4[1] = h128;
                hp4[(size_t)a.h16_lanes * 2] = h128;
                hp4[(size_t)a.h16_lanes * 2 + 1] = h128;
                if (a.znz) {
                    a.znz[(size_t)((p_hi - 32 + a.h16_shift) >> 4) * a.h16_lanes + p] = 0;
                    a.znz[(size_t)((p_hi - 16 + a.h16_shift) >> 4) * a.h16_lanes + p] = 0;
                }
                continue;
            }
        }
        // Coarse panel (reference mode, both sub-panels speculative): the far field with
        // the kOzCoarse most significant R digits, certified with the matching bound
        // (kRecCbC).  The weights of reference mode do not see the mean (the two squares
        // of ref_weight cancel to rounding), and the one-dominant-point margin of these
        // sigma_i ~ 1e-2 coordinates dwarfs the larger bound.
        bool coarse = false;
#ifndef LGS_NO_COARSE
        if constexpr (OZ && PB == 32 && !WL)
            coarse = p_hi >= 32 &&
                     __builtin_amdgcn_readfirstlane((int)((lds_cdptr)rec_lds)[31 * kRecStride + kRecSpec]) == 1 &&
                     __builtin_amdgcn_readfirstlane((int)((lds_cdptr)rec_lds)[15 * kRecStride + kRecSpec]) == 1;
#endif
        LGS_DC_T(t_far0);
        LGS_DC_ADD(0, t_far0 - t_panel0);
#ifdef LGS_DIAG_NO_FAR
        if (false) {
#else
        if (pk > 0) {
#endif
            // far field on the matrix cores; coefficients of rows >= p_hi were
            // stored by this wave's lanes in earlier panels
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
          if constexpr (OZ && PB == 32) {
            oz_far_field(a, pk, p_hi, p0, lane, (lds_cdptr)rec_lds, F, LDF, acc, ash, nzm, coarse);
            (void)NT;
          } else {
            d4_t f[NT][4];
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int g = 0; g < 4; ++g) f[t][g] = (d4_t){0.0, 0.0, 0.0, 0.0};
            // Stage s of step j0 covers columns jj = j0 + 4s: lane (kq, nq) reads
            // R rows 16t + nq at column jj + kq (RP panel block, PB doubles per
            // column) and the 4 coefficients of chains 4nq..4nq+3 at coordinate
            // jj + kq.  Uniform base pointers advance by one stage (4 columns);
            // the per-lane offsets are fixed.  Software pipeline, 4 stages deep:
            // the loads of step j0 + 16 are issued while the MFMAs of step j0
            // run; K = d - p_hi is a multiple of PB, so every step is full.
            const double* __restrict__ rbase = RP + (size_t)PB * PB * ((size_t)pk * (pk - 1) / 2);
            const ZT* __restrict__ zbase = Z + p0 + (size_t)p_hi * ldz;
            const size_t roff = (size_t)kq * PB + nq, zoff = (size_t)kq * ldz + 4 * nq;
            const size_t rstep = 4 * PB, zstep = 4 * ldz;
            double ra[4][NT];
            ZQuad<ZT> zq[4];
#pragma unroll
            for (int st = 0; st < 4; ++st) {
#pragma unroll
                for (int t = 0; t < NT; ++t) ra[st][t] = rbase[roff + 16 * t];
                zq[st].load(zbase + zoff);
                rbase += rstep;
                zbase += zstep;
            }
            auto consume = [&](int st) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const double bz = zq[st].get(g);
#pragma unroll
                    for (int t = 0; t < NT; ++t)
                        f[t][g] = __builtin_amdgcn_mfma_f64_16x16x4f64(ra[st][t], bz, f[t][g], 0, 0, 0);
                }
            };
            int j0 = p_hi;
            for (; j0 + 16 < d; j0 += 16) {
#pragma unroll
                for (int st = 0; st < 4; ++st) {
                    consume(st);
#pragma unroll
                    for (int t = 0; t < NT; ++t) ra[st][t] = rbase[roff + 16 * t];
                    zq[st].load(zbase + zoff);
                    rbase += rstep;
                    zbase += zstep;
                }
            }
#pragma unroll
            for (int st = 0; st < 4; ++st) consume(st);
            if constexpr (PB == 32) {
                // tile 1 (rows p_hi-16..p_hi-1) -> acc; tile 0 stays in LDS for the
                // second sub-panel
#pragma unroll
                for (int g = 0; g < 4; ++g)
#pragma unroll
                    for (int reg = 0; reg < 4; ++reg) F[(kq + 4 * reg) * LDF + 4 * nq + g] = f[1][g][reg];
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = F[r * LDF + lane];
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int g = 0; g < 4; ++g)
#pragma unroll
                    for (int reg = 0; reg < 4; ++reg) F[(kq + 4 * reg) * LDF + 4 * nq + g] = f[0][g][reg];
            } else {
                // D -> LDS [row][chain] -> one chain per lane, one 16-row tile at a time
#pragma unroll
                for (int t = 0; t < NT; ++t) {
#pragma unroll
                    for (int g = 0; g < 4; ++g)
#pragma unroll
                        for (int reg = 0; reg < 4; ++reg) F[(kq + 4 * reg) * LDF + 4 * nq + g] = f[t][g][reg];
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[16 * t + r] = F[r * LDF + lane];
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                }
            }
          }
        } else {
#pragma unroll
            for (int r = 0; r < NACC; ++r) acc[r] = 0.0;
            if constexpr (PB == 32) {
#pragma unroll
                for (int r = 0; r < 16; ++r) F[r * LDF + lane] = 0.0;
            }
        }
        LGS_DC_T(t_near0);
        LGS_DC_ADD(1, t_near0 - t_far0);
        if constexpr (PB == 32) {
            // Two-level near field: the 32-row panel is decided as two 16-row
            // sub-panels, so only 16 running sums are live across the SampleZ
            // calls (occupancy); the block R[L rows, U cols] that couples them is
            // applied with 16 MFMAs after the upper sub-panel U is decided.
            // Coefficients are kept in registers and stored once per sub-panel: a store
            // still in flight at a SampleZ call would be waited for at the callee's
            // entry (the calling convention starts with s_waitcnt 0).
            bool pnz = false;  // (OZ) a nonzero coefficient in this panel, this lane
#ifdef LGS_NEAR_UNROLLED  // the round-2 near field: 16 steps unrolled, SampleZ as leaf calls
            auto near16 = [&](int rows16, int top) __attribute__((always_inline)) {
                using ZH = std::conditional_t<sizeof(ZT) == 8, double, int>;
                ZH zh[16];
                cert_lds[1][threadIdx.x] = cert_lds[0][threadIdx.x];  // sum |z_j| before the sub-panel
                cert_lds[2][threadIdx.x] = lw;
#pragma unroll
                for (int s = 0; s < 16; ++s) {
                    if (s < rows16) {
                        const int i = __builtin_amdgcn_readfirstlane(top - 1 - s);
                        const lds_cdptr rec = (lds_cdptr)rec_lds + (i - (p_hi - 32)) * kRecStride;
                        // running sums rotate instead of shifting: logical acc[k] of step s
                        // lives in acc[(k - s) & 15] (s is a compile-time constant here), so
                        // no register moves per coordinate; 16 steps bring the map back
                        // Ca, Cb, c', 1/R_ii (record slots 21..24) in two 16-byte LDS reads
                        static_assert(kSzCa == 21 && kSzCb == 22 && kRecCp == 23 && kRecIrii == 24, "record layout");
                        typedef double d2v __attribute__((ext_vector_type(2)));
                        const RecRegs rr = load_rec(rec);
                        const double mu = (rr[kRecCp] - acc[(15 - s) & 15]) * rr[kRecIrii];
                        LGS_DC_T(t_sz0);
                        // certified decision at the blocked-order mean (the |z| sum
                        // bounded by the cap a.z1cap, checked after the sub-panel); a
                        // decision not covered is a guess, verified after the sub-panel
                        bool un;
                        const double zi = decide_coord_rec<WL, true, LIBM>(a, i, mu, rec, rr, rs, lw, flags, etab_s,
                                                                     cert_dmu(rr[kSzCa], rr[kSzCb], a.z1cap, mu),
                                                                     un, eb, tb);
                        if (un) cert_fl[threadIdx.x] |= 1 << s;
#ifdef LGS_DIAG_CYCLES
                        {
                            LGS_DC_T(t_sz1);
                            const int kind = (int)rec[2] & 7;
                            LGS_DC_ADD(3 + kind, t_sz1 - t_sz0);
                            LGS_DC_ADD(8 + kind, 1);
                        }
#endif
                        if constexpr (sizeof(ZT) == 8) {
                            zh[s] = zi;
                        } else {
                            if (sizeof(ZT) == 4 && !(zi <= 2147483647.0 && zi >= -2147483648.0))
                                flags |= kFlagOverflow;
                            if (sizeof(ZT) == 2 && !(zi <= 32767.0 && zi >= -32768.0)) flags |= kFlagOverflow16;
                            zh[s] = (int)fmin(fmax(zi, -2147483648.0), 2147483647.0);
                        }
                        if constexpr (OZ)
                            if (!(zi <= 32639.0 && zi >= -32767.0)) flags |= kFlagOverflow16;
#pragma unroll
                        for (int k = 0; k < 15; ++k) acc[(k - s) & 15] = fma(rr[kRecRs + 14 - k], zi, acc[(k - s) & 15]);
                        acc[(15 - s) & 15] = 0.0;  // the next step's logical acc[0]
                    }
                }
                // int16 history value (z + 128, clamped to the far field's digit range)
                auto hist_val = [&](int s) -> int {
                    if constexpr (sizeof(ZT) == 8)
                        return (int)(fmin(fmax(zh[s], -32767.0), 32639.0) + 128.0);
                    else
                        return min(max(zh[s], -32767), 32639) + 128;
                };
                // a whole sub-panel is one 16-coordinate history block ((top + shift) % 16
                // == 0; position 15 - s holds row top - 1 - s): two 16-byte stores
                const bool hblock = OZ && rows16 == 16;
#pragma unroll
                for (int s = 0; s < 16; ++s) {
                    if (s < rows16) {
                        const int i = top - 1 - s;
                        if constexpr (sizeof(ZT) == 8)
                            Z[(size_t)i * ldz + p] = (ZT)(int64_t)zh[s];
                        else
                            Z[(size_t)i * ldz + p] = (ZT)zh[s];
                        if constexpr (OZ) {  // int16 history (z + 128) for the int8-digit far field
                            if (!hblock) {
                                const int ih = i + a.h16_shift;
                                a.h16[((size_t)(ih >> 4) * a.h16_lanes + p) * 16 + (ih & 15)] = (int16_t)hist_val(s);
                            }
                            pnz |= zh[s] != 0;
                        }
                    }
                }
                if constexpr (OZ) {
                    if (hblock) {
                        v4u_t h[2];
#pragma unroll
                        for (int j = 0; j < 8; ++j)
                            h[j >> 2][j & 3] = ((unsigned int)hist_val(15 - 2 * j) & 0xffffu) |
                                               ((unsigned int)hist_val(14 - 2 * j) << 16);
                        v4u_t* hp = (v4u_t*)(a.h16 + ((size_t)((top - 16 + a.h16_shift) >> 4) * a.h16_lanes + p) * 16);
                        hp[0] = h[0];
                        hp[1] = h[1];
                    }
                }
                {
                    // the certificate used sum_{j>i} |z_j| <= z1cap: verify it (the sum at
                    // the sub-panel's end bounds every coordinate's) -- else replay
                    double z1e = cert_lds[1][threadIdx.x];  // (re-read: not live across the sub-panel)
#pragma unroll
                    for (int s = 0; s < 16; ++s)
                        if (s < rows16) z1e += fabs((double)zh[s]);
                    cert_lds[0][threadIdx.x] = z1e;
                }
                const int fl = cert_fl[threadIdx.x] | (cert_lds[0][threadIdx.x] > a.z1cap ? (1 << 16) : 0);
                if (__builtin_amdgcn_ballot_w64(fl != 0) != 0) {  // rare: verify / replay (whole wave)
                    cert_fl[threadIdx.x] = 0;
                    const int w64 = threadIdx.x & ~63;
                    const VerifyOut vo = verify_subpanel<WL, OZ>(kernel_args(), Z, ldz, p0, top, rows16, fl, lw,
                                                                 rs.step, rs.chain, &cert_lds[0][w64],
                                                                 &cert_lds[1][w64], &cert_lds[2][w64], flags);
                    lw = vo.lw;
                    flags = vo.flags;
                    if (WL) tb += vo.tabs;
                    if constexpr (OZ) pnz |= vo.nz != 0;
                }
                if constexpr (OZ)  // (this variant keeps no per-sub-panel flag: the block counts as nonzero)
                    if (a.znz) a.znz[(size_t)((top - 1 + a.h16_shift) >> 4) * a.h16_lanes + p] = 1;
            };
#endif
            // Rolled near field (default): one loop iteration per coordinate with the
            // decision inline -- no call in the hot path, so no SGPR spill / restore
            // around it, no wait-for-everything at a callee's entry, and the record
            // loads of the next steps can be scheduled under the current decision.
            // The running sums shift by one each step as part of the 15 FMAs
            // (acc[k + 1] = acc[k] + R[i-15+k][i] z_i, written in descending k, so in
            // place): acc[15] is always the current coordinate's sum.  z is stored per
            // step; the int16 history is packed into 8 registers (step s at position
            // 15 - s) and written as two 16-byte stores at the end.
            auto near16r = [&](int rows16, int top) __attribute__((always_inline)) {
                cert_lds[1][threadIdx.x] = cert_lds[0][threadIdx.x];  // sum |z_j| before the sub-panel
                cert_lds[2][threadIdx.x] = lw;
                double z1e = cert_lds[0][threadIdx.x];
#ifdef LGS_HIST_STORE16
                // (default) every coordinate's history value stored at once: the packing of a
                // whole sub-panel through 8 registers (8 VALU per coordinate) cost more than
                // the 16-bit store it saves (profiles/r05f_kb_trims.log)
                const bool hblock = false;
#else
                const bool hblock = OZ && rows16 == 16;
#endif
                unsigned int hp[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) hp[j] = 0u;
                int flm = 0;
#ifndef LGS_NO_CAP_SP
                // the whole sub-panel is capped with sigma >= 360 (host flag kRecSpec == 2):
                // its steps take the capped decision without the per-coordinate kind
                // dispatch (round 6, with the scheduler flags: C3 / C4 / C5 Klein -2.9 / -1.2
                // / -1.6 %, the bench 114.1 -> 116.8 M samples/s, identical hashes,
                // profiles/r06al_capsp.log; round 5, without them: neutral).  Such a
                // sub-panel is never in a coarse panel (two kRecSpec == 1 sub-panels), so
                // its certificate uses the sub-panel's own Cb.
                const int capsp = !LIBM && rows16 == 16 &&
                                  __builtin_amdgcn_readfirstlane((int)((lds_cdptr)rec_lds)[(top - 1 - (p_hi - 32)) * kRecStride + kRecSpec]) == 2;
#endif
                bool snz = false;  // (OZ) a nonzero z in this sub-panel, this lane
#ifdef LGS_TAIL3
                int izmx = 0, izmn = 0;  // (16-bit stores) the same extremes of the saturated int32 values
                int16_t* hptr = a.h16 + ((size_t)((top - 1 + a.h16_shift) >> 4) * a.h16_lanes + p) * 16 +
                                ((top - 1 + a.h16_shift) & 15);
#endif
#ifdef LGS_TAIL2
                double zmx = 0.0, zmn = 0.0;  // the sub-panel's largest / smallest z (range checks, snz)
                ZT* zrow = Z + (size_t)(top - 1) * ldz;  // row of the step's coordinate (uniform)
                const uint32_t zoff = (uint32_t)p * (uint32_t)sizeof(ZT);  // this lane's byte offset in a row
#endif
                double zsq = 0.0;  // (q-panel skip) sum z^2 of this sub-panel, this lane
#ifndef LGS_NEAR_UNROLL  // coordinates per loop iteration (the running sums shift by one per step)
#define LGS_NEAR_UNROLL 1
#endif
#pragma unroll LGS_NEAR_UNROLL
                for (int s = 0; s < rows16; ++s) {
#ifdef LGS_DIAG_STEP  // diagnostic builds only: phases of a near-field step (lgs_diag_cycles [3] [4] [5])
                    LGS_DC_T(t_stepA);
#endif
                    const int i = __builtin_amdgcn_readfirstlane(top - 1 - s);
                    const lds_cdptr rec = (lds_cdptr)rec_lds + (i - (p_hi - 32)) * kRecStride;
                    static_assert(kSzCa == 21 && kSzCb == 22 && kRecCp == 23 && kRecIrii == 24, "record layout");
#if defined(LGS_DBG1) || defined(LGS_PHILOX_TOP)
                    // (LGS_DBG1: the round-4 hazard reconstruction; LGS_PHILOX_TOP:
                    // the same placement as an optimisation) the coordinate's Philox block drawn
                    // under the record's LDS reads, off the decision's dependency chain
                    const RecRegs rr = load_rec(rec, [&]() { (void)rs.u((uint32_t)(d - 1 - i)); });
#elif defined(LGS_REC_SMEM)
                    const RecRegs rr = load_rec_g(cst(a.crec) + (size_t)i * kRecStride);
#elif defined(LGS_REC_RS_SMEM)
                    const RecRegs rr = load_rec(rec, cst(a.crec) + (size_t)i * kRecStride);
#else
                    const RecRegs rr = load_rec(rec);
#endif
                    const double mu = (rr[kRecCp] - acc[15]) * rr[kRecIrii];
                    LGS_DC_T(t_sz0);
                    bool un;
#ifndef LGS_NO_CAP_SP
                    int cf = __builtin_amdgcn_readfirstlane(capsp);
                    asm volatile("" : "+s"(cf));  // a scalar test per step (no loop unswitching: one copy of the loop)
                    const double zi = cf ? decide_capped_rec<WL>(a, i, mu, rec, rr, rs, lw, flags, etab_s,
                                                                 cert_dmu(rr[kSzCa], rr[kSzCb], a.z1cap, mu), un, eb, tb)
                                         : decide_coord_rec<WL, true, LIBM>(
                                               a, i, mu, rec, rr, rs, lw, flags, etab_s,
                                               cert_dmu(rr[kSzCa], coarse ? REC_CBC : rr[kSzCb], a.z1cap, mu), un,
                                               eb, tb);
#else
                    const double zi = decide_coord_rec<WL, true, LIBM>(
                        a, i, mu, rec, rr, rs, lw, flags, etab_s,
                        cert_dmu(rr[kSzCa], coarse ? REC_CBC : rr[kSzCb], a.z1cap, mu), un, eb, tb);
#endif
#ifdef LGS_TAIL3
                    if (__builtin_amdgcn_ballot_w64(un) != 0) flm |= un ? (1 << s) : 0;  // (rare)
#else
                    flm |= un ? (1 << s) : 0;
#endif
#if defined(LGS_DIAG_CYCLES) && !defined(LGS_DIAG_STEP)
                    {
                        LGS_DC_T(t_sz1);
                        const int kind = (int)rec[2] & 7;
                        LGS_DC_ADD(3 + kind, t_sz1 - t_sz0);
                        LGS_DC_ADD(8 + kind, 1);
                    }
#endif
#ifdef LGS_DIAG_STEP
                    LGS_DC_T(t_stepC);
#endif
                    // stores: v_cvt_i32_f64 saturates, so no clamps -- a value beyond the
                    // int16 history's range (or a 16-bit store's) flags kFlagOverflow16 and
                    // the launch is redone wider; beyond int32 is an error (kFlagOverflow)
#ifdef LGS_TAIL2
                    // (the range checks from the sub-panel's extremes after the loop; the store
                    // through the row's uniform base and a 32-bit lane offset)
#ifdef LGS_TAIL3
                    // 16-bit stores: the extremes of the saturated int32 conversion (one
                    // v_max_i32 / v_min_i32; fmax would canonicalise both operands first)
                    // detect every value outside the int16 / history range as well
                    const int zint = (int)zi;
                    if constexpr (sizeof(ZT) <= 2) {
                        izmx = max(izmx, zint);
                        izmn = min(izmn, zint);
                    } else {
                        zmx = fmax(zmx, zi);
                        zmn = fmin(zmn, zi);
                    }
#else
                    const int zint = (int)zi;
                    zmx = fmax(zmx, zi);
                    zmn = fmin(zmn, zi);
#endif
                    if constexpr (sizeof(ZT) == 8)
                        *(ZT*)((char*)zrow + zoff) = (ZT)(int64_t)zi;
                    else
                        *(ZT*)((char*)zrow + zoff) = (ZT)zint;
                    zrow -= ldz;
#else
                    if constexpr (sizeof(ZT) == 8) {
                        Z[(size_t)i * ldz + p] = (ZT)(int64_t)zi;
                    } else {
                        if (sizeof(ZT) == 4 && !(zi <= 2147483647.0 && zi >= -2147483648.0)) flags |= kFlagOverflow;
                        if (!OZ && sizeof(ZT) == 2 && !(zi <= 32767.0 && zi >= -32768.0)) flags |= kFlagOverflow16;
                        Z[(size_t)i * ldz + p] = (ZT)(int)zi;
                    }
#endif
                    if constexpr (OZ) {
#ifndef LGS_TAIL2
                        if (!(zi <= 32639.0 && zi >= -32767.0)) flags |= kFlagOverflow16;
#endif
                        // int16 history value z + 128 (exact whenever the range check passed)
                        const unsigned int hv = (unsigned int)((int)zi + 128) & 0xffffu;
                        if (hblock) {
#pragma unroll
                            for (int j = 7; j >= 1; --j) hp[j] = __builtin_amdgcn_alignbit(hp[j], hp[j - 1], 16);
                            hp[0] = (hp[0] << 16) | hv;
                        } else {
#ifdef LGS_TAIL3
                            // a sub-panel lies in one 16-coordinate history block ((top + shift)
                            // % 16 == 0): step s writes position 15 - s of this lane's block
                            *hptr = (int16_t)hv;
                            --hptr;
#else
                            const int ih = i + a.h16_shift;
                            a.h16[((size_t)(ih >> 4) * a.h16_lanes + p) * 16 + (ih & 15)] = (int16_t)hv;
#endif
                            if constexpr (!WL) zsq = fma(zi, zi, zsq);  // (whole sub-panels: from hp below)
                        }
#ifndef LGS_TAIL2
                        snz |= zi != 0.0;
#endif
                    }
                    // sum |z|: only the sub-panel's end reads it (the certificate's per-coordinate
                    // bound uses the cap), so a whole 16-row sub-panel takes it from the packed
                    // history below (exact: integers) -- kept in the loop, the compiler spilled
                    // it and its reload's vmcnt(0) waited for every coordinate's stores
                    if (!hblock) z1e += fabs(zi);
#pragma unroll
                    for (int k = 14; k >= 0; --k) acc[k + 1] = fma_shift(rr[kRecRs + 14 - k], zi, acc[k]);
                    acc[0] = 0.0;
#ifdef LGS_DIAG_STEP
                    {
                        LGS_DC_T(t_stepD);
                        LGS_DC_ADD(3, t_sz0 - t_stepA);  // record batch + mean
                        LGS_DC_ADD(4, t_stepC - t_sz0);  // decision (kind dispatch, Philox, SampleZ, weight)
                        LGS_DC_ADD(5, t_stepD - t_stepC);  // stores, history packing, bookkeeping, 15 FMAs
                        LGS_DC_ADD(8, 1);
                        LGS_DC_ADD(9, 1);
                        LGS_DC_ADD(10, 1);
                    }
#endif
                }
#ifdef LGS_TAIL3
                if constexpr (sizeof(ZT) <= 2) {
                    zmx = (double)izmx;
                    zmn = (double)izmn;
                }
#endif
#ifdef LGS_TAIL2
                if (sizeof(ZT) == 4 && !(zmx <= 2147483647.0 && zmn >= -2147483648.0)) flags |= kFlagOverflow;
                if (!OZ && sizeof(ZT) == 2 && !(zmx <= 32767.0 && zmn >= -32768.0)) flags |= kFlagOverflow16;
                if (OZ && !(zmx <= 32639.0 && zmn >= -32767.0)) flags |= kFlagOverflow16;
                if constexpr (OZ) snz = zmx != 0.0 || zmn != 0.0;
#endif
                if constexpr (OZ) {
                    if (hblock) {
                        v4u_t* hp4 = (v4u_t*)(a.h16 + ((size_t)((top - 16 + a.h16_shift) >> 4) * a.h16_lanes + p) * 16);
                        hp4[0] = (v4u_t){hp[0], hp[1], hp[2], hp[3]};
                        hp4[1] = (v4u_t){hp[4], hp[5], hp[6], hp[7]};
                        // sum |z| (and, reference mode, z^2) of the sub-panel from its packed
                        // history (z + 128; int16: signed)
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const double zl = (double)((int)(short)(hp[j] & 0xffffu) - 128);
                            const double zh = (double)((int)(short)(hp[j] >> 16) - 128);
                            z1e += fabs(zl) + fabs(zh);
                            if constexpr (!WL) {
                                zsq = fma(zl, zl, zsq);
                                zsq = fma(zh, zh, zsq);
                            }
                        }
                    }
                }
                // the certificate used sum_{j>i} |z_j| <= z1cap: verify it (the sum at the
                // sub-panel's end bounds every coordinate's) -- else replay
                cert_lds[0][threadIdx.x] = z1e;
                const int fl = flm | (z1e > a.z1cap ? (1 << 16) : 0);
                if (__builtin_amdgcn_ballot_w64(fl != 0) != 0) {  // rare: verify / replay (whole wave)
                    const int w64 = threadIdx.x & ~63;
                    const VerifyOut vo = verify_subpanel<WL, OZ>(kernel_args(), Z, ldz, p0, top, rows16, fl, lw,
                                                                 rs.step, rs.chain, &cert_lds[0][w64],
                                                                 &cert_lds[1][w64], &cert_lds[2][w64], flags);
                    lw = vo.lw;
                    flags = vo.flags;
                    if (WL) tb += vo.tabs;
                    if constexpr (OZ) snz |= vo.nz != 0;
                    if (vo.z2 >= 0.0) zsq = vo.z2;
                }
#ifndef LGS_NO_QSKIP_CODE
                if constexpr (OZ && !WL) {  // the q-panel skip's ||z_W||^2 (+inf: a speculative z != 0)
                    const bool spec_sp = rows16 == 16 &&
                                         __builtin_amdgcn_readfirstlane((int)((lds_cdptr)rec_lds)[(top - 1 - (p_hi - 32)) * kRecStride + kRecSpec]) == 1;
                    qzs[threadIdx.x] = spec_sp ? (zsq != 0.0 ? __builtin_inf() : qzs[threadIdx.x]) : qzs[threadIdx.x] + zsq;
                }
#endif
                if constexpr (OZ) {
                    pnz |= snz;
                    if (a.znz) a.znz[(size_t)((top - 1 + a.h16_shift) >> 4) * a.h16_lanes + p] = snz ? 1 : 0;
                    // the wave's 64-coordinate chunk of these rows holds a nonzero (B z skips
                    // the others with one word per 32 chunks, not one flag load per chunk)
#ifndef LGS_NO_CLIVE_K
                    if (a.clive && top >= 16 && __builtin_amdgcn_ballot_w64(snz) != 0 && lane == 0)
                        atomicOr(a.clive + (size_t)((top - 16) >> 11) * a.clive_ld + (p0 >> 6),
                                 1u << (((top - 16) >> 6) & 31));
#endif
                }
            };
            // one copy of the 16-step near field for both sub-panels (a second inlined
            // copy doubles the hot loop's code beyond the instruction cache)
            bool upper_zero = false;  // the upper sub-panel was kept speculatively: all its z are 0
#pragma nounroll
            for (int half = 0; half < 2; ++half) {
                const int top = p_hi - 16 * half;
                const int rows16 = top < 16 ? top : 16;
                if (rows16 <= 0) break;
                if (half == 1 && upper_zero) {
                    // the coupling R[L rows, U cols] z_U is exactly +0 (z_U = 0; the MFMA
                    // sums of +-0 products from +0 stay +0), and F + 0 = F: skip it
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[r] = F[r * LDF + lane];
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                } else if (half == 1) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    d4_t c[4];
#pragma unroll
                    for (int g = 0; g < 4; ++g) c[g] = (d4_t){0.0, 0.0, 0.0, 0.0};
                    const double* __restrict__ rx = a.rx + (size_t)pk * 256 + lane;
                    const ZT* __restrict__ zu = Z + p0 + (size_t)(p_hi - 16) * ldz + (size_t)kq * ldz + 4 * nq;
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk) {
                        const double av = rx[64 * kk];
                        ZQuad<ZT> q;
#ifdef LGS_DIAG_COUPLE_NOLOAD  // diagnostic builds only (NOT bit-exact): the coupling without its Z reload
                        q.load(Z + p0 + 4 * nq);
#else
                        q.load(zu + (size_t)(4 * kk) * ldz);
#endif
#pragma unroll
                        for (int g = 0; g < 4; ++g)
                            c[g] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, q.get(g), c[g], 0, 0, 0);
                    }
#pragma unroll
                    for (int g = 0; g < 4; ++g)
#pragma unroll
                        for (int reg = 0; reg < 4; ++reg) F[(kq + 4 * reg) * LDF + 4 * nq + g] += c[g][reg];
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[r] = F[r * LDF + lane];
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                }
#ifndef LGS_NO_SPEC
                // Speculative sub-panel (host flag kRecSpec: 16 coordinates of the small
                // kind, e.g. the q-coordinates of NTRU / q-ary bases, whose sigma_i ~ 1e-2
                // make z = rint(mu) = 0 all but always): decided all at once assuming every
                // earlier z of the sub-panel is 0.  With those z = 0 the sequential form's
                // FMAs leave the running sums bit-for-bit unchanged (fma(r, +-0, a) = a; a
                // is never -0), so each mean -- hence each decision and weight term -- is
                // exactly the sequential one.  Kept only when every lane's 16 decisions are
                // certified one-dominant-point decisions (no draw) with z = 0; otherwise the
                // sub-panel is redone sequentially from the untouched sums.
                if (rows16 == 16 &&
                    __builtin_amdgcn_readfirstlane(
                        (int)((lds_cdptr)rec_lds)[(top - 1 - (p_hi - 32)) * kRecStride + kRecSpec]) == 1) {
                    double term[16];
                    // the bound dmu assumes sum_{j>i} |z_j| <= z1cap; with every z of the
                    // sub-panel 0 that sum is the one at its start (else: the sequential
                    // path, whose end-of-sub-panel check verifies)
                    bool ok = cert_lds[0][threadIdx.x] <= a.z1cap;
                    double ebs = 0.0;  // (WL) the sub-panel's weight bound
#pragma unroll
                    for (int s = 0; s < 16; ++s) {
                        const lds_cdptr rec = (lds_cdptr)rec_lds + (top - 1 - s - (p_hi - 32)) * kRecStride;
                        const double mu = (rec[kRecCp] - acc[15 - s]) * rec[kRecIrii];
                        const double is = rec[1], is2 = is * is;
                        const double c = rint(mu), d1 = fabs(mu - c), t = d1 * is;
                        const double emax = -0.5 * (t * t);
                        const double gap = 0.5 * is2 * (1.0 - 2.0 * d1);
                        const double hl = ceil(mu + rec[6]) - floor(mu - rec[6]);
                        const double dmu = cert_dmu(rec[kSzCa], coarse ? rec[kRecCbC] : rec[kSzCb], a.z1cap, mu);
                        const bool fast = gap > 745.2 && !(a.linear_probs && emax < -745.2) &&
                                          gap - 745.2 > 1.01 * dmu * hl * is2 + 1e-12 * gap;
                        ok = ok && isfinite(mu) && fast && c == 0.0;
                        term[s] = WL ? emax : ref_weight(c, mu, rec[kRecRos], rec[kRecIsr], rec[kRecLterm]);
                        if (WL) ebs += wl_bound_dominant(emax, is2, d1, dmu);
                    }
                    if (__builtin_amdgcn_ballot_w64(!ok) == 0) {
#pragma unroll
                        for (int s = 0; s < 16; ++s) lw += term[s];  // the sequential order
                        if (WL) {
#pragma unroll
                            for (int s = 0; s < 16; ++s) tb += fabs(term[s]);
                            eb += ebs;
                        }
#pragma unroll
                        for (int s = 0; s < 16; ++s) Z[(size_t)(top - 1 - s) * ldz + p] = (ZT)0;
                        if constexpr (OZ) {  // int16 history: z + 128 in all 16 positions
                            v4u_t* hp4 = (v4u_t*)(a.h16 + ((size_t)((top - 16 + a.h16_shift) >> 4) * a.h16_lanes + p) * 16);
                            hp4[0] = (v4u_t){0x00800080u, 0x00800080u, 0x00800080u, 0x00800080u};
                            hp4[1] = (v4u_t){0x00800080u, 0x00800080u, 0x00800080u, 0x00800080u};
                        }
                        if (OZ && a.znz) a.znz[(size_t)((top - 1 + a.h16_shift) >> 4) * a.h16_lanes + p] = 0;
                        upper_zero = true;
                        continue;
                    }
                }
#endif
#ifdef LGS_NEAR_UNROLLED
                near16(rows16, top);
#else
                near16r(rows16, top);
#endif
            }
            if constexpr (OZ) {  // visible to the block at the next panel's staging barrier
                if (__builtin_amdgcn_ballot_w64(pnz) != 0 && lane == 0) atomicOr(&nzm[pk >> 5], 1u << (pk & 31));
            }
            LGS_DC_T(t_near1);
            LGS_DC_ADD(2, t_near1 - t_near0);
        } else {
            for (int s = 0; s < rows; ++s) {
                const int i = p_hi - 1 - s;
                const double mu = (cst(a.cp)[i] - acc[PB - 1]) * cst(a.irii)[i];
                double zi = decide_coord<WL>(a, i, mu, rs, lw, flags, etab_s,
                                             cert_dmu(cst(a.cert)[2 * i], cst(a.cert)[2 * i + 1], z1, mu), eb, tb);
                if (zi == kAmbiguous) zi = resolve_coord<WL>(a, i, Z + p, ldz, rs, lw, flags, tb);
                z1 += fabs(zi);
                store_z(Z, (size_t)i * ldz + p, zi, flags);
                const double x = zi;
                const cdptr rc = cst(RC) + (size_t)i * (PB - 1);
#pragma unroll
                for (int k = 0; k < PB - 1; ++k) acc[k] = fma(rc[PB - 2 - k], x, acc[k]);
#pragma unroll
                for (int k = PB - 1; k >= 1; --k) acc[k] = acc[k - 1];
                acc[0] = 0.0;
            }
        }
    }
    if constexpr (PB == 32) {  // the largest sum |z_j| of the wave -> the context's cap
        double m = active ? cert_lds[0][threadIdx.x] : 0.0;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m = fmax(m, __shfl_xor(m, o));
        if (lane == 0 && a.z1max) atomicMax(a.z1max, (unsigned long long)__double_as_longlong(m));
    }
    const double ewl = WL ? wl_bound_sum(eb, tb, d) : 0.0;
    if (WL && PB == 32 && a.emax) {  // the wave's largest weight bound -> the context's running maximum
        double m = active ? ewl : 0.0;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m = fmax(m, __shfl_xor(m, o));
        if (lane == 0) atomicMax(a.emax, (unsigned long long)__double_as_longlong(m));
    }
    if (!active) return;
    if (a.LW) a.LW[p] = lw;
    if (WL && PB == 32 && a.LWE) a.LWE[p] = ewl;
    if (WL && PB != 32) wl_bound_store(a, p, ewl);
    if (flags) atomicOr(a.flags, flags);
#ifdef LGS_DIAG_CYCLES
    LGS_DC_T(t_kernel1);
    dc[13] = t_kernel1 - t_kernel0;
    if (lane == 0)
        for (int k = 0; k < 16; ++k) atomicAdd(&lgs_diag_cycles[k], (unsigned long long)dc[k]);
#endif
}

// ------------------------------------------------------------ log density
// compute_log_density (klein.py:222-271) of given coefficient vectors, reference
// arithmetic order: sum_i -0.5*((z_i-mu_i)/sigma_i)^2 - (0.5*log(2pi) + log sigma_i)
// - log_Z_i, where log_Z_i = logsumexp of the already-normalised table is 0 up to
// rounding (taken as 0).
template <typename ZT>
__global__ __launch_bounds__(256) void log_density_kernel(const KleinArgs a,
                                                          const double* __restrict__ R,
                                                          const ZT* __restrict__ Z,
                                                          double* __restrict__ out) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.n) return;
    const int d = a.d;
    const size_t ldz = (size_t)a.ldz;
    double lp = 0.0;
    for (int i = d - 1; i >= 0; --i) {
        const double* __restrict__ Ri = R + (size_t)i * d;
        double cs = 0.0;
        for (int j = i + 1; j < d; ++j) cs = cs + Ri[j] * (double)Z[(size_t)j * ldz + p];
        const double mu = (a.cp[i] - cs) / a.rii[i];
        const double t = ((double)Z[(size_t)i * ldz + p] - mu) / a.sig_ref[i];
        lp += -0.5 * (t * t);
        lp -= a.lterm[i];
    }
    out[p] = lp;
}

// ------------------------------------------------------------ SampleZ probe
// Direct evaluation of the device SampleZ for given (mu, sigma, u) triples
// (unit test / diagnostics of klein.py:101-179's decision).
__global__ __launch_bounds__(256) void samplez_probe_kernel(const double* __restrict__ mu,
                                                            const double* __restrict__ sig,
                                                            const double* __restrict__ u,
                                                            int64_t n, int precision,
                                                            int linear, int mode, const double* __restrict__ etab,
                                                            int64_t* __restrict__ z,
                                                            double* __restrict__ ln) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    // mode 0: sample_z with log-normaliser; 1: table walk; 2: decision only.
    const SampleZOut o = mode == 1 ? sample_z_table(mu[p], sig[p], precision, linear != 0, u[p])
                                   : sample_z(mu[p], sig[p], precision, linear != 0, u[p],
                                              mode == 0, etab);
    z[p] = o.z;
    if (ln) ln[p] = o.log_norm;
}

// ------------------------------------------------------------ IMHK accept
// One lane per chain; proposals of step t for chain c live at p = c*T + t
// (chain-major, so the kept states of a chain are contiguous columns).
// sel[c*n_keep + k] = proposal index of the state retained after step
// (k+1)*thin (-1 = the carried-in state); cnt[p] / cnt_carry[c] count the
// retained steps spent in each state (moments), final_sel[c] = last state.
__device__ __forceinline__ bool aborted(const unsigned int* abort) {
    return abort && (*(const volatile unsigned int*)abort & kAbortMask) != 0u;
}
// need: a device-gated replay (lgs_imhk without a host wait on B z) runs only when
// the int8-digit B z before it flagged a coefficient beyond its digits
__device__ __forceinline__ bool not_needed(const unsigned int* need) {
    return need && (*(const volatile unsigned int*)need & kFlagI8Range) == 0u;
}

__global__ __launch_bounds__(256) void imhk_accept_kernel(const AcceptArgs a) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.nc || aborted(a.abort)) return;
    double lw_x = a.lw_state[c];
    int64_t cur = -1;
    int64_t acc = 0;
    int64_t keep = 0;
    int32_t carry = 0;
    const uint32_t chain = a.chain0 + (uint32_t)c;
    for (int64_t t = 0; t < a.T; ++t) {
        const int64_t p = c * a.T + t;
        const double lw_y = a.LW[p];
        double ratio;
        if (lw_x == -INFINITY) {
            ratio = 1.0;
        } else {
            const double r = exp(lw_y - lw_x);
            ratio = r < 1.0 ? r : 1.0;  // min(1.0, r); NaN -> 1.0 like Python's min
        }
        const double u = accept_uniform(a.seed, a.step0 + (uint32_t)t, chain);
        const bool take = u < ratio;
        if (take) {
            cur = p;
            lw_x = lw_y;
            ++acc;
        }
        if (a.acc_step) a.acc_step[c * a.acc_ld + t] = take ? 1 : 0;
        if ((t + 1) % a.thin == 0) {
            if (a.lw_keep) a.lw_keep[c * a.lw_ld + keep] = lw_x;
            if (a.sel) a.sel[c * a.n_keep + keep] = cur >= 0 ? cur : (a.carry_col >= 0 ? a.carry_col + c : -1);
            if (a.cnt) {
                if (cur < 0)
                    ++carry;
                else
                    a.cnt[cur] += 1;
            }
            ++keep;
        }
    }
    a.lw_state[c] = lw_x;
    a.accepts[c] += acc;
    a.final_sel[c] = cur;
    if (a.cnt_carry) a.cnt_carry[c] = carry;
    if (a.state_init && cur >= 0) a.state_init[c] = init_code(a.step0 + (uint32_t)(cur % a.T));
}

// ------------------------------------------------- certified Wang-Ling decisions
// The blocked kernels' Wang-Ling weights are within LWE of the reference-order
// values (wl_bound_*).  A decision u < min(1, exp(lw_y - lw_x)) (imhk.py:158-167) is
// taken at those weights only when it is the same for every pair within the
// bounds; otherwise the wave recomputes both weights in the reference's order
// (wl_exact_wave) and decides at them -- the decision klein_exact_kernel's weights
// give.  Chain states carried into a block have the bound *emax (the context's
// running maximum over its Wang-Ling draws); one that has to be recomputed is
// replayed with its own counters when its state_init word records the step it was
// drawn at (the chain's draws are counter-addressed, so the replay is the
// reference-order weight of that draw, checked to reproduce its z), else with step
// 0's uniforms (they only select SampleZ's rare table-walk path, whose normaliser
// agrees to ~1e-13) and a residual bound 1e-12 (1 + |lw|).  Certification covers
// states drawn in this context since its last lgs_set_basis (EMAX is reset there).

__device__ __forceinline__ double readlane_f64(double v, int k) {
    const long long b = __double_as_longlong(v);
    return __longlong_as_double(((long long)__builtin_amdgcn_readlane((int)(b >> 32), k) << 32) |
                                (unsigned int)__builtin_amdgcn_readlane((int)b, k));
}
__device__ __forceinline__ double zload(const void* base, int zb, int64_t off) {
    if (zb == 2) return (double)((const int16_t*)base)[off];
    if (zb == 4) return (double)((const int32_t*)base)[off];
    return (double)((const int64_t*)base)[off];
}

// decide_coord's draw and Wang-Ling term at mean mu, for a coordinate i that may
// differ between lanes (global-pointer SampleZ constants: no uniformisation)
__device__ __forceinline__ double wl_decide_lane(const KleinArgs& a, int i, double mu, double u, double& ln) {
    ln = 0.0;
    if (!isfinite(mu)) return 0.0;
    const double s = a.szc ? a.szc[(size_t)i * kSzcStride] : a.sig[i];
    if (s == 0.0) return rint(mu);
    if (a.szc)
        return sample_z_coord(mu, u, (gdptr)(a.szc + (size_t)i * kSzcStride), a.precision, a.linear_probs != 0,
                              true, (gdptr)a.etab, ln, -1.0);
    const SampleZOut o = sample_z(mu, s, a.precision, a.linear_probs != 0, u, true, a.etab);
    ln = o.log_norm;
    return (double)o.z;
}

// Wang-Ling log weight of ONE sample in the reference's arithmetic order -- what
// klein_exact_kernel returns for it: the means (c'_i - sum_{j>i} R_ij z_j) / R_ii
// with the j-ascending unfused sum of klein.py:191-195, each coordinate's window
// normaliser at its mean (decide_coord's SampleZ call, same uniform), added for
// i = d-1 .. 0.  Whole wave, uniform arguments.  Lane k owns coordinates k + 64 m
// (16 per pass, so d > 1024 takes several passes, top rows first); z_j is broadcast
// (zero terms skipped: cs + R * (+-0) = cs, cs is never -0), R is read through its
// transpose (one coalesced row segment per m).  z_j at zsrc[j * zst], width zb.
// check: the draws at those means must reproduce z (the sample's own counters).
__device__ double wl_exact_wave(const KleinArgs& a, const double* __restrict__ RT, const void* zsrc, int zb,
                                int64_t zst, uint32_t step, uint32_t chain, bool check, int& bad) {
    const int lane = threadIdx.x & 63;
    const int d = a.d;
    constexpr int MB = 16;
    const int M = (d + 63) / 64;
    CoordStreamT<false> rs;
    rs.init(a.seed, step, chain);
    double lw = 0.0;
    for (int mb = (M - 1) / MB * MB; mb >= 0; mb -= MB) {
        const int ilo = 64 * mb;
        double cs[MB];
#pragma unroll
        for (int m = 0; m < MB; ++m) cs[m] = 0.0;
        for (int j0 = ilo; j0 < d; j0 += 64) {
            const double zv = j0 + lane < d ? zload(zsrc, zb, (int64_t)(j0 + lane) * zst) : 0.0;
            const int jn = min(64, d - j0);
            for (int k = 0; k < jn; ++k) {
                const double zj = readlane_f64(zv, k);
                if (zj == 0.0) continue;
                const int j = j0 + k;
                const double* __restrict__ rt = RT + (size_t)j * d + ilo + lane;
#pragma unroll
                for (int m = 0; m < MB; ++m)
                    if (ilo + 64 * m + lane < j) cs[m] = cs[m] + rt[64 * m] * zj;
            }
        }
        double lnv[MB];
#pragma unroll
        for (int m = 0; m < MB; ++m) {
            const int i = ilo + 64 * m + lane;
            lnv[m] = 0.0;
            if (i < d) {
                const double mu = (a.cp[i] - cs[m]) / a.rii[i];
                const double zi = wl_decide_lane(a, i, mu, rs.u((uint32_t)(d - 1 - i)), lnv[m]);
                if (check && zi != zload(zsrc, zb, (int64_t)i * zst)) bad = 1;
            }
        }
#pragma unroll
        for (int m = MB - 1; m >= 0; --m) {
            if (ilo + 64 * m >= d) continue;
            for (int k = 63; k >= 0; --k)
                if (ilo + 64 * m + k < d) lw = lw + readlane_f64(lnv[m], k);
        }
    }
    return lw;
}

__device__ __forceinline__ double accept_ratio(double lw_y, double lw_x) {
    if (lw_x == -INFINITY) return 1.0;
    const double r = exp(lw_y - lw_x);
    return r < 1.0 ? r : 1.0;  // min(1.0, r); NaN -> 1.0 like Python's min
}
// true when u < min(1, exp(lw_y' - lw_x')) is the same for every |lw_x' - lw_x| <= e_x,
// |lw_y' - lw_y| <= e_y (take: the decision).  The difference of the two computed
// differences is <= e_x + e_y + 2u(|lw_x| + |lw_y|); exp is monotone to within its
// ~1 ulp error (the 1e-15 factors).
__device__ __forceinline__ bool accept_certain(double lw_x, double e_x, double lw_y, double e_y, double u,
                                               bool& take) {
    take = u < accept_ratio(lw_y, lw_x);
    if (e_x == 0.0 && e_y == 0.0) return true;
    if (!isfinite(lw_x) || !isfinite(lw_y)) return false;
    const double D = lw_y - lw_x;
    const double eps = e_x + e_y + 2.3e-16 * (fabs(lw_x) + fabs(lw_y));
    const double rlo = fmin(1.0, exp(D - eps) * (1.0 - 1e-15));
    const double rhi = fmin(1.0, exp(D + eps) * (1.0 + 1e-15));
    return u < rlo || u >= rhi;
}

// imhk_accept_kernel with certified decisions (AcceptArgs.LWE non-null): one wave
// per block, every lane stays to the end (the rare recomputation needs the whole
// wave); lanes beyond nc write nothing.
__global__ __launch_bounds__(64) void imhk_accept_cert_kernel(const AcceptArgs a, const KleinArgs ka) {
    if (aborted(a.abort)) return;
    const int lane = threadIdx.x & 63;
    const int64_t c0 = (int64_t)blockIdx.x * 64;
    const int64_t c = c0 + lane;
    const bool live = c < a.nc;
    double lw_x = live ? a.lw_state[c] : 0.0;
    double e_x = a.bscale * __longlong_as_double((long long)*(const volatile unsigned long long*)a.emax);
    const int32_t sinit = live && a.state_init ? a.state_init[c] : 1;  // the carried state's draw
    int64_t cur = -1;
    int64_t acc = 0;
    int64_t keep = 0;
    int32_t carry = 0;
    unsigned int nres = 0;
    int bad = 0;
    const uint32_t chain = a.chain0 + (uint32_t)c;
    for (int64_t t = 0; t < a.T; ++t) {
        const int64_t p = c * a.T + t;
        double lw_y = live ? a.LWx[p] : 0.0;
        double e_y = live ? a.bscale * a.LWE[p] : 0.0;
        const double u = accept_uniform(a.seed, a.step0 + (uint32_t)t, chain);
        bool take = false;
        const bool sure = !live || accept_certain(lw_x, e_x, lw_y, e_y, u, take);
        uint64_t todo = __builtin_amdgcn_ballot_w64(!sure);
        while (todo) {  // rare: reference-order weights of lane L's proposal and state
            const int L = __builtin_ctzll(todo);
            todo &= todo - 1;
            const int64_t cL = c0 + L;
            const uint32_t chL = a.chain0 + (uint32_t)cL;
            const double eyL = readlane_f64(e_y, L), exL = readlane_f64(e_x, L);
            const int64_t curL = ((int64_t)__builtin_amdgcn_readlane((int)(cur >> 32), L) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)cur, L);
            const int32_t sinitL = __builtin_amdgcn_readlane(sinit, L);
            double ly = 0.0, lx = 0.0;
            int badx = 0;  // (the carried state's replay did not reproduce its z)
            if (eyL != 0.0)
                ly = wl_exact_wave(ka, a.RT, (const char*)a.Zst + (cL * a.T + t) * a.zb, a.zb, a.ldz,
                                   a.step0 + (uint32_t)t, chL, true, bad);
            if (exL != 0.0) {
                if (curL >= 0)  // an earlier proposal of this block
                    lx = wl_exact_wave(ka, a.RT, (const char*)a.Zst + curL * a.zb, a.zb, a.ldz,
                                       a.step0 + (uint32_t)(curL % a.T), chL, true, bad);
                else  // the state carried in: replayed at its own step when state_init has it
                    lx = wl_exact_wave(ka, a.RT,
                                       (const char*)a.zs + (a.zs_cm ? cL : cL * ka.d) * a.ob, a.ob,
                                       a.zs_cm ? a.nc : 1,
                                       sinitL >= kInitStep0 ? (uint32_t)(sinitL - kInitStep0) : 0u, chL,
                                       sinitL >= kInitStep0, badx);
            }
            bad |= badx;
            // a carried state replayed without its counters keeps a residual bound -- and so
            // does one whose recorded step did not reproduce it (drawn under
            // another seed or chain mapping, e.g. a resume with another seed)
            const bool resid = exL != 0.0 && curL < 0 &&
                               (sinitL < kInitStep0 || __builtin_amdgcn_ballot_w64(badx != 0) != 0);
            if (lane == L) {
                if (eyL != 0.0) {
                    lw_y = ly;
                    e_y = 0.0;
                    a.LWx[p] = ly;
                    a.LWE[p] = 0.0;
                }
                if (exL != 0.0) {
                    lw_x = lx;
                    e_x = resid ? 1e-12 * (1.0 + fabs(lx)) : 0.0;
                    if (cur >= 0) {
                        a.LWx[cur] = lx;
                        a.LWE[cur] = 0.0;
                    }
                }
                take = u < accept_ratio(lw_y, lw_x);
                ++nres;
            }
        }
        if (!live) continue;
        if (take) {
            cur = p;
            lw_x = lw_y;
            e_x = e_y;
            ++acc;
        }
        if (a.acc_step) a.acc_step[c * a.acc_ld + t] = take ? 1 : 0;
        if ((t + 1) % a.thin == 0) {
            if (a.lw_keep) a.lw_keep[c * a.lw_ld + keep] = lw_x;
            if (a.sel) a.sel[c * a.n_keep + keep] = cur >= 0 ? cur : (a.carry_col >= 0 ? a.carry_col + c : -1);
            if (a.cnt) {
                if (cur < 0)
                    ++carry;
                else
                    a.cnt[cur] += 1;
            }
            ++keep;
        }
    }
    if (nres) atomicAdd(a.flagw + kFlagWordAcceptResolved, nres);
    if (__builtin_amdgcn_ballot_w64(bad != 0) != 0 && lane == 0) atomicAdd(a.flagw + kFlagWordWLMismatch, 1u);
    if (!live) return;
    a.lw_state[c] = lw_x;
    a.accepts[c] += acc;
    a.final_sel[c] = cur;
    if (a.cnt_carry) a.cnt_carry[c] = carry;
    if (a.state_init && cur >= 0) a.state_init[c] = init_code(a.step0 + (uint32_t)(cur % a.T));
}

// ------------------------------------------------------------ moments
// Moments of the retained states and the chains' final states in one pass over
// the proposal store: mom[i] += sum_p cnt[p] z[i][p], mom[d+i] += sum_p cnt[p]
// z[i][p]^2, and where final_sel[p / T] == p (fsel non-null) the value is also the
// chain's new state, written to z_state in the caller's layout -- the final-state
// gather folded into the pass that already reads every proposal (a separate
// gather touches one proposal in T per cache line).  VEC: 8 (16-bit store) or 4
// consecutive proposals per lane in one load (ldz and n multiples of that).
// RY coordinates per workgroup (vector path): the weights cnt and the chains'
// final-state indices are loaded once for RY rows of the store instead of once
// per row (they were 2-3x the coefficient bytes per row, from L2).
template <typename ZT, typename OT, bool VEC, int RY = 1, bool GS = false>
__global__ __launch_bounds__(256) void moments_final_kernel(const ZT* __restrict__ Z, int64_t ldz,
                                                            const int32_t* __restrict__ cnt, int64_t n,
                                                            int64_t T, const int64_t* __restrict__ fsel,
                                                            int d, int64_t chunk,
                                                            unsigned long long* mom,
                                                            OT* __restrict__ zs, int zs_cm, int64_t nc,
                                                            const unsigned int* abort,
                                                            const uint8_t* __restrict__ znz, int64_t zlanes,
                                                            int zshift, const unsigned int* need) {
    if (aborted(abort) || not_needed(need)) return;
    __shared__ long long r1[RY][4], r2[RY][4];
    auto tile = [&](const int i0, const int64_t p0) {
    const int64_t p1 = p0 + chunk < n ? p0 + chunk : n;
    long long s1[RY], s2[RY];
#pragma unroll
    for (int r = 0; r < RY; ++r) s1[r] = s2[r] = 0;
    auto put = [&](int i, int64_t c, long long z) {
        if (zs_cm)
            zs[(size_t)i * nc + c] = (OT)z;
        else
            zs[(size_t)c * d + i] = (OT)z;
    };
    if constexpr (VEC) {
        // VW consecutive proposals per lane in one 16-byte load (8 for a 16-bit store)
        constexpr int VW = sizeof(ZT) == 2 ? 8 : 4;
        typedef ZT zv_t __attribute__((ext_vector_type(VW)));
        typedef int iv4_t __attribute__((ext_vector_type(4)));
        const double rT = 1.0 / (double)T;
        // (znz: the Klein launch's per-(16-coordinate block, proposal) nonzero flags; the
        // VW proposals of a load whose blocks are all zero need no coefficient load)
        const int zb0 = (i0 + zshift) >> 4, zb1 = (i0 + RY - 1 + zshift) >> 4;
        for (int64_t p = p0 + VW * (int64_t)threadIdx.x; p < p1; p += VW * 256) {
            zv_t zv[RY];
            bool live = true;
            if (znz != nullptr) {
                typedef unsigned int u2_t __attribute__((ext_vector_type(2)));
                const u2_t f0 = *(const u2_t*)(znz + (size_t)zb0 * zlanes + p);
                const u2_t f1 = *(const u2_t*)(znz + (size_t)zb1 * zlanes + p);
                live = ((f0[0] | f0[1] | f1[0] | f1[1]) != 0u);
            }
#pragma unroll
            for (int r = 0; r < RY; ++r)
                zv[r] = live && i0 + r < d ? *(const zv_t*)(Z + (size_t)(i0 + r) * ldz + p) : (zv_t){};
            int w[VW];
#pragma unroll
            for (int g = 0; g < VW / 4; ++g) {
                const iv4_t wv = cnt ? *(const iv4_t*)(cnt + p + 4 * g) : (iv4_t){1, 1, 1, 1};
#pragma unroll
                for (int k = 0; k < 4; ++k) w[4 * g + k] = wv[k];
            }
#pragma unroll
            for (int r = 0; r < RY; ++r)
#pragma unroll
                for (int k = 0; k < VW; ++k) {
                    if constexpr (sizeof(ZT) == 2) {  // z^2 < 2^30: one 32x32->64 multiply-add each
                        const int z = zv[r][k];
                        s1[r] += (long long)w[k] * z;
                        s2[r] += (long long)w[k] * (z * z);
                    } else {
                        const long long z = zv[r][k];
                        s1[r] += w[k] * z;
                        s2[r] += w[k] * z * z;
                    }
                }
            if (fsel) {  // chains whose proposals touch [p, p + VW - 1] (one, two at a boundary)
                // p / T through the fp64 reciprocal, corrected by one step (p < 2^32)
                int64_t c = (int64_t)((double)p * rT);
                const int64_t rem = p - c * T;
                c += rem < 0 ? -1 : (rem >= T ? 1 : 0);
                for (; c * T <= p + VW - 1 && c < nc; ++c) {
                    const int64_t k = fsel[c] - p;
#pragma unroll
                    for (int e = 0; e < VW; ++e)
                        if (k == e)
#pragma unroll
                            for (int r = 0; r < RY; ++r)
                                if (i0 + r < d) put(i0 + r, c, (long long)zv[r][e]);
                }
            }
        }
    } else {
        const ZT* __restrict__ zr = Z + (size_t)i0 * ldz;
        for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
            const long long z = (long long)zr[p], w = cnt ? cnt[p] : 1;
            s1[0] += w * z;
            s2[0] += w * z * z;
            if (fsel) {
                const int64_t c = (int64_t)((uint32_t)p / (uint32_t)T);  // n < 2^32 (checked by the caller)
                if (fsel[c] == p) put(i0, c, z);
            }
        }
    }
    // wave sums by shuffles, then the 4 waves' partials through LDS
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int r = 0; r < RY; ++r) {
        long long a = s1[r], b = s2[r];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            a += __shfl_xor(a, o);
            b += __shfl_xor(b, o);
        }
        if (lane == 0) {
            r1[r][wave] = a;
            r2[r][wave] = b;
        }
    }
    __syncthreads();
    if ((int)threadIdx.x < RY && i0 + (int)threadIdx.x < d) {
        const int r = threadIdx.x;
        atomicAdd(mom + i0 + r, (unsigned long long)(r1[r][0] + r1[r][1] + r1[r][2] + r1[r][3]));
        atomicAdd(mom + d + i0 + r, (unsigned long long)(r2[r][0] + r2[r][1] + r2[r][2] + r2[r][3]));
    }
    };
    if constexpr (GS) {  // grid-strided: the gated fallback after B z's moments launches a small grid
        const int64_t nbx = (n + chunk - 1) / chunk;
        const int nby = (d + RY - 1) / RY;
        for (int by = blockIdx.y; by < nby; by += gridDim.y)
            for (int64_t bx = blockIdx.x; bx < nbx; bx += gridDim.x) {
                tile(by * RY, bx * chunk);
                __syncthreads();  // (r1 / r2 reused by the next tile)
            }
    } else {
        tile(blockIdx.y * RY, (int64_t)blockIdx.x * chunk);
    }
}

// Carried-in states (row-major or coordinate-major z_state) weighted by cnt_carry.
template <typename ZT>
__global__ __launch_bounds__(256) void moments_carry_kernel(const ZT* __restrict__ zs,
                                                            int coord_major, int64_t nc, int d,
                                                            const int32_t* __restrict__ cc,
                                                            unsigned long long* mom,
                                                            const unsigned int* abort,
                                                            const unsigned int* need) {
    if (aborted(abort) || not_needed(need)) return;
    for (int i = blockIdx.x; i < d; i += gridDim.x) {
    long long s1 = 0, s2 = 0;
    for (int64_t c = threadIdx.x; c < nc; c += blockDim.x) {
        const long long w = cc[c];
        if (!w) continue;
        const long long z = (long long)(coord_major ? zs[(size_t)i * nc + c] : zs[(size_t)c * d + i]);
        s1 += w * z;
        s2 += w * z * z;
    }
    __shared__ long long r1[256], r2[256];
    r1[threadIdx.x] = s1;
    r2[threadIdx.x] = s2;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            r1[threadIdx.x] += r1[threadIdx.x + o];
            r2[threadIdx.x] += r2[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        atomicAdd(mom + i, (unsigned long long)r1[0]);
        atomicAdd(mom + d + i, (unsigned long long)r2[0]);
    }
    __syncthreads();  // (r1 / r2 reused by the next strided coordinate)
    }
}

// ------------------------------------------------------------ gathers
// Retained / final states: out row q (d coefficients) = src column sel[q] of Z,
// or row q of the carried state zs when sel[q] < 0.  Thread per (i, q), q fastest.
template <typename ZT, typename OT>
__global__ __launch_bounds__(256) void gather_z_kernel(const ZT* __restrict__ Z, int64_t ldz,
                                                       const int64_t* __restrict__ sel,
                                                       int64_t nq, int64_t q_per_chain,
                                                       const OT* __restrict__ zs,
                                                       int zs_coord_major, int64_t nc, int d,
                                                       OT* __restrict__ out, int out_coord_major,
                                                       const unsigned int* abort) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    if (q >= nq || aborted(abort)) return;
    const int64_t s = sel[q];
    OT v;
    if (s >= 0) {
        v = (OT)Z[(size_t)i * ldz + s];
    } else {
        const int64_t c = q / q_per_chain;
        v = zs_coord_major ? zs[(size_t)i * nc + c] : zs[(size_t)c * d + i];
    }
    if (out_coord_major)
        out[(size_t)i * nq + q] = v;
    else
        out[(size_t)q * d + i] = v;
}

// Sets kFlagOverflow16 when a coefficient does not fit a 16-bit store (the chain
// states a 16-bit proposal store receives through carry_cols).
template <typename OT>
__global__ __launch_bounds__(256) void range16_kernel(const OT* __restrict__ zs, int64_t count,
                                                      unsigned int* flags) {
    bool out = false;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < count;
         e += (int64_t)gridDim.x * blockDim.x)
        out |= zs[e] > (OT)32767 || zs[e] < (OT)-32768;
    if (out) atomicOr(flags, kFlagOverflow16);
}

// Chain states (caller layout, width OT) into columns col0 .. col0+nc-1 of the
// coordinate-major proposal store, so kept-state selections are plain columns.
template <typename OT, typename ZT>
__global__ __launch_bounds__(256) void carry_cols_kernel(const OT* __restrict__ zs, int zs_coord_major,
                                                         int64_t nc, int d, ZT* __restrict__ Z,
                                                         int64_t ldz, int64_t col0, unsigned int* flags) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    if (c >= nc) return;
    const OT v = zs_coord_major ? zs[(size_t)i * nc + c] : zs[(size_t)c * d + i];
    if (sizeof(ZT) == 2 && flags && (v > (OT)32767 || v < (OT)-32768)) atomicOr(flags, kFlagCarry16);
    Z[(size_t)i * ldz + col0 + c] = (ZT)v;
}

// Initial IMHK draws without a host round trip (lgs_imhk): *any = some chain has
// init == 0; then each such chain takes its proposal (column c of Z) and weight.
__global__ __launch_bounds__(256) void uninit_scan_kernel(const int32_t* __restrict__ init, int64_t nc,
                                                          unsigned int* any) {
    bool u = false;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nc; c += (int64_t)gridDim.x * blockDim.x)
        u |= init[c] == 0;
    if (__builtin_amdgcn_ballot_w64(u) != 0 && (threadIdx.x & 63) == 0) atomicOr(any, 1u);
}

template <typename ZT, typename OT>
__global__ __launch_bounds__(256) void init_apply_kernel(const ZT* __restrict__ Z, int32_t* __restrict__ init,
                                                         int64_t nc, int d, const double* __restrict__ LW,
                                                         OT* __restrict__ zs, int zs_cm, double* __restrict__ lws,
                                                         unsigned int* flags) {
    const bool ab = aborted(flags);
    // the verification count so far (the initial draws'), kept if the block's own
    // Klein launch is discarded
    if (blockIdx.x == 0 && threadIdx.x == 0) flags[kFlagWordCheckpoint] = ab ? 0u : flags[kFlagWordResolved];
    if (flags[kFlagWordUninit] == 0u || ab) return;
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nc || init[c] != 0) return;
    for (int i = 0; i < d; ++i) {
        const OT v = (OT)Z[(size_t)i * nc + c];
        if (zs_cm)
            zs[(size_t)i * nc + c] = v;
        else
            zs[(size_t)c * d + i] = v;
    }
    lws[c] = LW[c];
    init[c] = kInitStep0;  // the draw at counter step 0
}

// Z[coord][p] (ld ldz) -> out[p][coord] (row-major n x d), 64x64 tiles via LDS.
template <typename ZT, typename OT>
__global__ __launch_bounds__(256) void transpose_kernel(const ZT* __restrict__ Z, int64_t ldz,
                                                        int64_t n, int d, OT* __restrict__ out) {
    __shared__ OT tile[64][65];
    const int64_t p0 = (int64_t)blockIdx.x * 64;
    const int i0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int i = i0 + r;
        const int64_t p = p0 + tx;
        if (i < d && p < n) tile[r][tx] = (OT)Z[(size_t)i * ldz + p];
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
        const int64_t p = p0 + r;
        const int i = i0 + tx;
        if (i < d && p < n) out[(size_t)p * d + i] = tile[tx][r];
    }
}

// Row-major int z (n x d) -> coordinate-major Z[coord][p] (ld ldz).
template <typename ZT, typename IT>
__global__ __launch_bounds__(256) void to_coord_major_kernel(const IT* __restrict__ in, int64_t n,
                                                             int d, ZT* __restrict__ Z,
                                                             int64_t ldz) {
    __shared__ ZT tile[64][65];
    const int64_t p0 = (int64_t)blockIdx.x * 64;
    const int i0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int64_t p = p0 + r;
        const int i = i0 + tx;
        if (i < d && p < n) tile[r][tx] = (ZT)in[(size_t)p * d + i];
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
        const int i = i0 + r;
        const int64_t p = p0 + tx;
        if (i < d && p < n) Z[(size_t)i * ldz + p] = tile[tx][r];
    }
}

// ------------------------------------------------------------ B z (fp64 MFMA)
// V[s][r] = sum_c B[r][c] Z[c][s] for s in [0, n), r in [0, d).
// Block tile 64 samples x 64 coords, 4 waves in 2x2, each wave 2x2 MFMA tiles of
// v_mfma_f64_16x16x4_f64 (A: lane l -> A[l&15][l>>4]; B: B[l>>4][l&15];
// D: row (l>>4)+4*reg, col l&15).  K staged through LDS in chunks of 16.
// Exact (bit-identical to any summation order) when B and z are integers and
// |partial sums| < 2^53.
template <typename ZT>
__global__ __launch_bounds__(256) void bz_gemm_kernel(const ZT* __restrict__ Z, int64_t ldz,
                                                      const int64_t* __restrict__ sel,
                                                      const double* __restrict__ BT, int d,
                                                      int64_t n, double* __restrict__ V,
                                                      int64_t ldv, int64_t rb, int64_t rstride,
                                                      int64_t roff, const unsigned int* abort,
                                                      const unsigned int* need) {
    if (aborted(abort) || not_needed(need)) return;  // (whole grid) the selections were not written
    constexpr int BM = 64, BN = 64, KC = 16, LDP = 80;  // LDP: padded row (doubles)
    __shared__ double As[KC][LDP];
    __shared__ double Bs[KC][LDP];
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    // row and sample tiles strided over the grid (one per workgroup except in the gated
    // replay's small grid, which must not cost a full-size dispatch when not needed:
    // beside a running Klein launch every workgroup waits for a free slot)
    for (int r0 = blockIdx.y * BN; r0 < d; r0 += gridDim.y * BN)
    for (int64_t s0 = (int64_t)blockIdx.x * BM; s0 < n; s0 += (int64_t)gridDim.x * BM) {
    d4_t acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = (d4_t){0.0, 0.0, 0.0, 0.0};
    for (int c0 = 0; c0 < d; c0 += KC) {
#pragma unroll
        for (int e = 0; e < (KC * BM) / 256; ++e) {
            const int idx = tid + 256 * e;
            const int kk = idx / BM, m = idx % BM;
            const int c = c0 + kk;
            const int64_t s = s0 + m;
            As[kk][m] = (c < d && s < n) ? (double)Z[(size_t)c * ldz + (sel ? sel[s] : s)] : 0.0;
            const int r = r0 + m;
            Bs[kk][m] = (c < d && r < d) ? BT[(size_t)c * d + r] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int k4 = 0; k4 < KC; k4 += 4) {
            const int kk = k4 + (lane >> 4);
            double af[2], bf[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                af[t] = As[kk][wm * 32 + t * 16 + (lane & 15)];
                bf[t] = Bs[kk][wn * 32 + t * 16 + (lane & 15)];
            }
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const int64_t s = s0 + wm * 32 + a * 16 + (lane >> 4) + 4 * reg;
                const int r = r0 + wn * 32 + b * 16 + (lane & 15);
                if (s < n && r < d) {
                    const int64_t row = (s / rb) * rstride + roff + s % rb;
                    V[(size_t)row * ldv + r] = acc[a][b][reg];
                }
            }
    }
}

// ------------------------------------------------------------ B z, exact int8 MFMA
// For integer bases with |B| <= 32639 and coefficients |z| <= 32639 the lattice
// points are computed exactly with two balanced base-256 digits per operand
// (x = 256 x1 + x0, x0, x1 in [-128, 127]) on v_mfma_i32_32x32x32_i8:
//   v = 65536 * (B1 z1) + 256 * (B1 z0 + B0 z1) + B0 z0,
// three int32 accumulators (|partial| <= 2 d 2^14 < 2^31 for d <= 65536),
// combined in int64 and converted to fp64 (exact below 2^53).  A coefficient out
// of range sets kFlagI8Range and the host recomputes with the fp64 kernel.
// Block tile 64 samples x 128 coords, K chunks of 64 through LDS; waves 2x2, each
// 32 samples x 64 coords = two 32x32 MFMA tiles.  Operand maps (32x32x32 i8):
// A row / B column = lane & 31, 16 consecutive k per lane (k = 16*(lane>>5) + j;
// any k permutation shared by A and B gives the same sum); D: col = lane & 31,
// row = (reg & 3) + 8*(reg >> 2) + 4*(lane >> 5).
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v16i_t __attribute__((ext_vector_type(16)));

// a 64-bit value rotated within each 16-lane DPP row (CTRL = 0x120 + r: row_ror:r)
template <int CTRL>
__device__ __forceinline__ unsigned long long dpp_row_ror_u64(unsigned long long x) {
    const unsigned int lo = (unsigned int)__builtin_amdgcn_update_dpp(0, (int)(unsigned int)x, CTRL, 0xf, 0xf, false);
    const unsigned int hi = (unsigned int)__builtin_amdgcn_update_dpp(0, (int)(unsigned int)(x >> 32), CTRL, 0xf, 0xf, false);
    return ((unsigned long long)hi << 32) | lo;
}

#ifndef LGS_BZ_OCC
#define LGS_BZ_OCC 3  // (round 5: pinned to three workgroups per CU; unpinned the int32 store instantiation drifted to 174 VGPRs)
#endif
#ifndef LGS_BZ_TXPER
#define LGS_BZ_TXPER 1
#endif
#ifndef LGS_BZ_TA
#define LGS_BZ_TA 1
#endif
template <typename ZT>
__global__ __launch_bounds__(256, LGS_BZ_OCC) void bz_i8_kernel(const ZT* __restrict__ Z, int64_t ldz,
                                                    const int64_t* __restrict__ sel,
                                                    const int* __restrict__ kchunk,
                                                    const int* __restrict__ koff,
                                                    const int8_t* __restrict__ Bd1,
                                                    const int8_t* __restrict__ Bd0, int dc, int d,
                                                    int64_t n, double* __restrict__ V, int64_t ldv,
                                                    int64_t rb, int64_t rstride, int64_t roff,
                                                    unsigned int* flags, int tx_count, int64_t ty_count,
                                                    const int16_t* __restrict__ h16, int64_t h16_lanes,
                                                    int64_t hcols, const unsigned int* abort,
                                                    const uint8_t* __restrict__ znz,
                                                    const unsigned int* __restrict__ clive, int64_t clive_ld,
                                                    double* __restrict__ VNP, int64_t vn_n,
                                                    unsigned long long* __restrict__ MP, int64_t mp_ld,
                                                    unsigned int* __restrict__ MPL) {
    if (aborted(abort)) return;  // (whole grid) the selections were not written
    constexpr int TA = LGS_BZ_TA;  // 32-sample MFMA tiles per wave
    constexpr int BM = 64 * TA, BN = kBzBN, KC = 64, P = 80;  // P: LDS row pitch (bytes), conflict-free
    constexpr int TN = BN / 64;  // 32-coordinate MFMA tiles per wave (waves 2 x 2)
    constexpr int KPT = KC * BM / 256;  // coefficients per thread per chunk
    __shared__ __attribute__((aligned(16))) int8_t Zs1[BM * P], Zs0[BM * P], Bs1[BN * P], Bs0[BN * P];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    // XCD-aware tile order: workgroups are dealt round-robin to the 8 XCDs, so
    // workgroup b runs on XCD b % 8; the tx_count coordinate tiles of one sample
    // tile are given to consecutive workgroups of the same XCD, which then reads
    // that sample tile's coefficients from HBM once and from its own L2 after.
    // Each workgroup computes LGS_BZ_TXPER consecutive coordinate tiles of its
    // sample tile, so the output stores of one tile drain while the MFMAs of the
    // next one run.
    const int64_t b = blockIdx.x, w = b >> 3;
    const int64_t ty = (w / tx_count) * 8 + (b & 7);
    const int txg = (int)(w % tx_count);
    if (ty >= ty_count) return;
    const int64_t s0 = ty * BM;
    const int ntx = (d + BN - 1) / BN;
    ZT zmax = 0, zmin = 0;  // range of the coefficients read (exactness check)
    for (int tx = txg * LGS_BZ_TXPER; tx < ntx && tx < (txg + 1) * LGS_BZ_TXPER; ++tx) {
    const int r0 = tx * BN;
    v16i_t p1[TA][TN], p2[TA][TN], p3[TA][TN];
#pragma unroll
    for (int ta = 0; ta < TA; ++ta)
#pragma unroll
        for (int t = 0; t < TN; ++t) {
            p1[ta][t] = (v16i_t){};
            p2[ta][t] = (v16i_t){};
            p3[ta][t] = (v16i_t){};
        }
    const int zm = tid & (BM - 1), zq = tid / BM;
    const int64_t zs_ = s0 + zm;
    const int64_t zcol = zs_ < n ? (sel ? sel[zs_] : zs_) : 0;  // this thread's sample column
    // only the K chunks where this row tile of B has a non-zero digit (exact skip)
    // (the block-sparsity lists are per 128-row tile of B)
    const int ci0 = koff[tx * BN / 128];
#ifdef LGS_DIAG_BZ_NOMFMA  // diagnostic builds only: epilogue cost probe
    const int ci1 = ci0;
#else
    const int ci1 = koff[tx * BN / 128 + 1];
#endif
    // Chunks where every sample of the tile has z = 0 on all 64 coordinates contribute
    // exactly nothing: skipped.  The Klein launch that wrote the history flags each
    // (16-coordinate block, sample) holding a nonzero (znz); thread (zm, zq) checks
    // block zq of each chunk for its sample, the tile ORs them in LDS.  Samples read
    // from the coefficient store (not that launch's) count as nonzero.  (NTRU / q-ary
    // bases: the q-coordinates' z are 0, which leaves ~1 of 6 chunks per tile.)
    // (round 4) the Klein launch also leaves, per wave, one bit per 64-coordinate chunk
    // (clive): the tile's live chunks are the OR of its samples' waves' words -- one
    // load per 32 chunks and sample instead of one flag load and LDS atomic per chunk
    const bool use_clive = KPT == 16 && h16 != nullptr && clive != nullptr;
    const bool use_znz = !use_clive && KPT == 16 && h16 != nullptr && znz != nullptr;
    __shared__ unsigned int livew[kOzMaxD / 64 / 32];
    // (round 5) every wave ORs the words itself: the 4 waves hold the same 64 samples
    // (zm = lane), so no LDS round trip and barrier precede the first chunk's loads;
    // the word stays in a scalar register up to d = 2048, else in the wave's LDS row
    __shared__ unsigned int livew4[4][kOzMaxD / 64 / 32];
    const int ngw = (d + 2047) / 2048;
    unsigned int live1 = 0u;
    if (use_clive) {
        {
            const int ng = ngw;
#ifndef LGS_BZ_NO_GUESS
            // the word of the identity selection (row q = proposal q: every kept state a
            // fresh proposal, e.g. acceptance 1) is loaded beside the selection itself
            // instead of after it; a lane whose selection differs reloads
            const int64_t zg = zs_ < n ? zs_ : 0;
            const unsigned int wg0 = zg < hcols ? clive[zg >> 6] : 0xffffffffu;
            const bool same = (zcol >> 6) == (zg >> 6) && (zcol < hcols) == (zg < hcols);
#endif
            for (int g = 0; g < ng; ++g) {
                unsigned int w = 0u;
#ifndef LGS_BZ_NO_GUESS
                const unsigned int wg =
                    g == 0 ? wg0 : (zg < hcols ? clive[(size_t)g * clive_ld + (zg >> 6)] : 0xffffffffu);
                if (zs_ < n)
                    w = same ? wg : (zcol < hcols ? clive[(size_t)g * clive_ld + (zcol >> 6)] : 0xffffffffu);
#else
                if (zs_ < n) w = zcol < hcols ? clive[(size_t)g * clive_ld + (zcol >> 6)] : 0xffffffffu;
#endif
                // OR over the wave's lanes; all equal (the tile's samples from one Klein
                // wave) needs no shuffles
                const unsigned int w0 = __builtin_amdgcn_readfirstlane(w);
                if (__builtin_amdgcn_ballot_w64(w != w0) != 0ull) {
#pragma unroll
                    for (int o = 32; o >= 1; o >>= 1) w |= __shfl_xor(w, o);
                } else {
                    w = w0;
                }
                if (ng == 1)
                    live1 = __builtin_amdgcn_readfirstlane(w);
                else if (lane == 0)
                    livew4[wave][g] = w;
            }
            if (ng > 1) {  // the wave's own LDS row: in order within the wave
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
    }
    // (MP) the tile's live-chunk words for the moments' reduction: a chunk the tile
    // skips leaves its partials unwritten
    if (MP != nullptr && use_clive && tx == 0 && tid < ngw) MPL[(size_t)ty * ngw + tid] = ngw == 1 ? live1 : livew4[0][tid];
    if (use_znz) {
        const bool hp = zs_ < n && zcol < hcols;
        for (int w = tid; w < (ci1 - ci0 + 31) / 32; w += 256) livew[w] = 0u;
        __syncthreads();
        for (int ci = ci0; ci < ci1; ++ci) {
            const int c0 = (kchunk[ci] & 0xffff) * KC;
            const bool nz = zs_ < n && (!hp || znz[(size_t)((c0 + zq * 16) >> 4) * h16_lanes + zcol] != 0);
            if (nz) atomicOr(&livew[(ci - ci0) >> 5], 1u << ((ci - ci0) & 31));
        }
        __syncthreads();
    }
    for (int ci = ci0; ci < ci1; ++ci) {
        // (bit 16 of a chunk entry: this row tile owns the chunk's moments, MP)
        const int kraw = kchunk[ci];
        const int cix = kraw & 0xffff;
        const bool mown = MP != nullptr && (kraw >> 16) != 0 && KPT == 16 && (BN == 128 || (tx & 1) == 0);
        if ((use_clive && !(((ngw == 1 ? live1 : livew4[wave][cix >> 5]) >> (cix & 31)) & 1u)) ||
            (use_znz && !((livew[(ci - ci0) >> 5] >> ((ci - ci0) & 31)) & 1u))) {  // (uniform)
            continue;  // (an all-zero chunk's moment partials stay 0: MP is cleared per launch)
        }
        const int c0 = cix * KC;
        if (KPT == 16 && h16 != nullptr && zs_ < n && zcol < hcols) {
            // column written by the Klein launch whose int16 history (z + 128,
            // [coordinate / 16][lane][16]) holds this sample's 16 coefficients in 32
            // contiguous bytes: the digit planes are byte permutes of them (exact:
            // that launch checked |z| against the history's range)
            const v4u_t* hp = (const v4u_t*)(h16 + ((size_t)((c0 + zq * 16) >> 4) * h16_lanes + zcol) * 16);
            const v4u_t y0 = hp[0], y1 = hp[1];
            v4i_t w0, w1;
            w1[0] = (int)__builtin_amdgcn_perm(y0[1], y0[0], 0x07050301u);
            w1[1] = (int)__builtin_amdgcn_perm(y0[3], y0[2], 0x07050301u);
            w1[2] = (int)__builtin_amdgcn_perm(y1[1], y1[0], 0x07050301u);
            w1[3] = (int)__builtin_amdgcn_perm(y1[3], y1[2], 0x07050301u);
            w0[0] = (int)(__builtin_amdgcn_perm(y0[1], y0[0], 0x06040200u) ^ 0x80808080u);
            w0[1] = (int)(__builtin_amdgcn_perm(y0[3], y0[2], 0x06040200u) ^ 0x80808080u);
            w0[2] = (int)(__builtin_amdgcn_perm(y1[1], y1[0], 0x06040200u) ^ 0x80808080u);
            w0[3] = (int)(__builtin_amdgcn_perm(y1[3], y1[2], 0x06040200u) ^ 0x80808080u);
            *(v4i_t*)&Zs0[zm * P + zq * 16] = w0;
            *(v4i_t*)&Zs1[zm * P + zq * 16] = w1;
        } else {  // z chunk -> balanced base-256 digits, [sample][k] byte planes
            const bool sok = zs_ < n;
            const ZT* zp = Z + (size_t)(c0 + zq * KPT) * ldz + zcol;
#pragma unroll
            for (int h = 0; h < KPT / 16; ++h) {
            v4i_t w0, w1;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                // z = 256 hi + lo with lo in [-128, 127]: lo's byte is z's low
                // byte and hi = (z + 128) >> 8, whose byte is byte 1 of z + 128;
                // v_perm_b32 gathers four such bytes into one dword
                unsigned int zz[4], hh[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int c = c0 + zq * KPT + h * 16 + q * 4 + j;
                    const ZT zr = (sok && c < d) ? zp[(size_t)(h * 16 + q * 4 + j) * ldz] : (ZT)0;
                    zmax = max(zmax, zr);
                    zmin = min(zmin, zr);
                    zz[j] = (unsigned int)(int)zr;
                    hh[j] = zz[j] + 128u;
                }
                w0[q] = (int)(__builtin_amdgcn_perm(zz[1], zz[0], 0x0c0c0400u) |
                              __builtin_amdgcn_perm(zz[3], zz[2], 0x04000c0cu));
                w1[q] = (int)(__builtin_amdgcn_perm(hh[1], hh[0], 0x0c0c0501u) |
                              __builtin_amdgcn_perm(hh[3], hh[2], 0x05010c0cu));
            }
            *(v4i_t*)&Zs0[zm * P + zq * KPT + h * 16] = w0;
            *(v4i_t*)&Zs1[zm * P + zq * KPT + h * 16] = w1;
            }
        }
#pragma unroll
        for (int e = 0; e < BN / 64; ++e) {  // B digit planes [coord][k], 16 B per thread per plane
            const int idx = tid + 256 * e;
            const int row = idx >> 2, part = idx & 3;
            const size_t g = (size_t)(r0 + row) * dc + c0 + part * 16;
            *(v4i_t*)&Bs1[row * P + part * 16] = *(const v4i_t*)&Bd1[g];
            *(v4i_t*)&Bs0[row * P + part * 16] = *(const v4i_t*)&Bd0[g];
        }
        __syncthreads();
        auto moment_partials = [&]() __attribute__((always_inline)) {
            // (round 5) the kept states' moments ride on this tile's digit planes while the
            // MFMAs run (round 6: called after the chunk's MFMAs are issued, so the VALU work
            // runs under the matrix pipe -- with the 16-byte stores below, B z 7.19 -> 6.98 ms
            // per 2^22 lattice points, profiles/r06q_bz_ab.log; LGS_BZ_MOM_EARLY: ahead of
            // them): wave w sums coordinates 16w..16w+15 of the chunk over the tile's 64
            // rows, lane (4 coordinates: lane >> 4) x (4 rows: lane & 15), packed per row as
            // z^2 * 2^24 + (z + 32768) (64 rows: the low field < 2^22, the total < 2^63;
            // rows past n hold z = 0 and add the bias only), then over the 16 lanes of a
            // DPP row (row_ror 8, 4, 2, 1: VALU moves, no LDS round trip)
            const int kk = 16 * wave + 4 * (lane >> 4);
            unsigned long long ps[4] = {0ull, 0ull, 0ull, 0ull};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = 4 * (lane & 15) + i;
                const unsigned int lo4 = *(const unsigned int*)&Zs0[row * P + kk];
                const unsigned int hi4 = *(const unsigned int*)&Zs1[row * P + kk];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int z = 256 * (int)(signed char)(hi4 >> (8 * j)) + (int)(signed char)(lo4 >> (8 * j));
                    ps[j] += ((unsigned long long)(unsigned int)(z * z) << 24) + (unsigned int)(z + 32768);
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                ps[j] += dpp_row_ror_u64<0x128>(ps[j]);  // row_ror:8
                ps[j] += dpp_row_ror_u64<0x124>(ps[j]);  // row_ror:4
                ps[j] += dpp_row_ror_u64<0x122>(ps[j]);  // row_ror:2
                ps[j] += dpp_row_ror_u64<0x121>(ps[j]);  // row_ror:1
            }
            if ((lane & 15) == 0) {
                unsigned long long* mp = MP + (size_t)ty * mp_ld + c0 + kk;
#pragma unroll
                for (int j = 0; j < 4; ++j) mp[j] = ps[j];
            }
        };
#ifdef LGS_BZ_MOM_EARLY
        if (mown) moment_partials();
#endif
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int kb = ks * 32 + 16 * (lane >> 5);
            v4i_t a1[TA], a0[TA];
#pragma unroll
            for (int ta = 0; ta < TA; ++ta) {
                const int arow = (wm * TA + ta) * 32 + (lane & 31);
                a1[ta] = *(const v4i_t*)&Zs1[arow * P + kb];
                a0[ta] = *(const v4i_t*)&Zs0[arow * P + kb];
            }
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int col = wn * (BN / 2) + tn * 32 + (lane & 31);
                const v4i_t b1 = *(const v4i_t*)&Bs1[col * P + kb];
                const v4i_t b0 = *(const v4i_t*)&Bs0[col * P + kb];
#pragma unroll
                for (int ta = 0; ta < TA; ++ta) {
                    p1[ta][tn] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1[ta], b1, p1[ta][tn], 0, 0, 0);
                    p2[ta][tn] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1[ta], b0, p2[ta][tn], 0, 0, 0);
                    p2[ta][tn] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0[ta], b1, p2[ta][tn], 0, 0, 0);
                    p3[ta][tn] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0[ta], b0, p3[ta][tn], 0, 0, 0);
                }
            }
        }
#ifndef LGS_BZ_MOM_EARLY
        if (mown) moment_partials();
#endif
        __syncthreads();
    }
    // output rows: sample q -> (q / rb) * rstride + roff + q % rb.  The wave's 32
    // rows start at qb (wave-uniform); with rb >= 32 they cross at most one block
    // boundary, so each row's address is a uniform base + row * ldv + (one
    // uniform jump past the boundary) -- no per-row division or 64-bit multiply.
    // v = 65536 p1 + 256 p2 + p3 is formed in fp64: every partial sum is an
    // integer below 2^53, so it is exact (and equal to the int64 combination).
    const int lrow = 4 * (lane >> 5);
#pragma unroll
    for (int ta = 0; ta < TA; ++ta) {
    const int64_t qb = s0 + (wm * TA + ta) * 32;
    if (VNP && qb < vn_n) {
        // ||v||^2 of the tile's rows (a scalar functional of the kept states, SURVEY
        // 8e): one partial sum per (row, 64-coordinate half tile), stored to its own
        // slot VNP[(2 tx + wn) vn_n + q] and summed per row by vnorm2_reduce_kernel (atomics
        // on the 64 rows' few cache lines from 16 workgroups serialised: 0.5 ms per 2^20).
        // Only the rows q < vn_n (the leading chains a lag series follows): computed for
        // every row this epilogue cost 0.94 ms per 2^20 (bz 1.70 -> 2.65 ms).
        // Lane & 31 is the coordinate: the 16 rows' partial sums are reduced over the 32
        // lanes by halving (16 shuffles instead of 80).  Integral v: exact in any order.
        double vs[16];
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            vs[reg] = 0.0;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
                if (r0 + wn * (BN / 2) + tn * 32 + (lane & 31) < d) {
                    const double v = fma((double)p1[ta][tn][reg], 65536.0, (double)p2[ta][tn][reg] * 256.0) +
                                     (double)p3[ta][tn][reg];
                    vs[reg] = fma(v, v, vs[reg]);
                }
        }
        int ridx = 0;
#pragma unroll
        for (int half = 8; half >= 1; half >>= 1) {  // lane bit 16 -> 8 values, bit 8 -> 4, ...
            const int bit = half * 2;
            const bool up = (lane & bit) != 0;
#pragma unroll
            for (int j = 0; j < half; ++j) {
                const double send = up ? vs[j] : vs[j + half];
                const double keep = up ? vs[j + half] : vs[j];
                vs[j] = keep + __shfl_xor(send, bit);
            }
            ridx += up ? half : 0;
        }
        const double tot = vs[0] + __shfl_xor(vs[0], 1);
        const int row = (ridx & 3) + 8 * (ridx >> 2) + lrow;
        const int64_t q = qb + row;
        if (!(lane & 1) && q < vn_n) VNP[(size_t)(2 * tx + wn) * vn_n + q] = tot;
    }
    const int64_t cb = qb / rb;
    const int64_t kb0 = qb - cb * rb;
    const int nrow = (int)min<int64_t>(n - qb, 32);  // valid rows of this tile
#ifndef LGS_BZ_NARROW
    // (round 6, with the moments after the MFMAs: B z 7.19 -> 6.98 ms per 2^22 lattice
    // points, profiles/r06q_bz_ab.log) 16-byte stores: lanes 2c and 2c + 1 swap one value per pair of rows
    // (DPP quad_perm [1, 0, 3, 2]), so the even lane holds row r, columns 2c and 2c + 1
    // and the odd lane row r + 1, the same columns (even d and ldv, V 16-byte aligned: every
    // pair then starts on a 16-byte boundary; otherwise the 8-byte stores below)
    if (rb >= 32 && (d & 1) == 0 && (ldv & 1) == 0 && ((uintptr_t)V & 15) == 0) {
        typedef double v2d_t __attribute__((ext_vector_type(2)));
        const int wrap_row = (int)min<int64_t>(rb - kb0, 32);
        const bool odd = (lane & 1) != 0;
        const int c = r0 + wn * (BN / 2) + ((lane & 31) & ~1);
        double* const vbase = V + (size_t)(cb * rstride + roff + kb0) * ldv + c;
        const int64_t jump = (rstride - rb) * ldv;
#pragma unroll
        for (int reg = 0; reg < 16; reg += 2) {
            const int row = (reg & 3) + 8 * (reg >> 2) + lrow + (odd ? 1 : 0);
            double* vrow = vbase + (size_t)row * ldv + (row >= wrap_row ? jump : 0);
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const double va = fma((double)p1[ta][tn][reg], 65536.0, (double)p2[ta][tn][reg] * 256.0) +
                                  (double)p3[ta][tn][reg];
                const double vb = fma((double)p1[ta][tn][reg + 1], 65536.0, (double)p2[ta][tn][reg + 1] * 256.0) +
                                  (double)p3[ta][tn][reg + 1];
                const double send = odd ? va : vb;
                const unsigned long long sb = __double_as_longlong(send);
                const unsigned int rlo = (unsigned int)__builtin_amdgcn_mov_dpp((int)(unsigned int)sb, 0xb1, 0xf, 0xf, false);
                const unsigned int rhi = (unsigned int)__builtin_amdgcn_mov_dpp((int)(unsigned int)(sb >> 32), 0xb1, 0xf, 0xf, false);
                const double recv = __longlong_as_double((long long)(((unsigned long long)rhi << 32) | rlo));
                v2d_t o;
                o[0] = odd ? recv : va;
                o[1] = odd ? vb : recv;
                if (row < nrow && c + tn * 32 < d) __builtin_nontemporal_store(o, (v2d_t*)(vrow + tn * 32));
            }
        }
    } else
#endif
    if (rb >= 32) {
        const int wrap_row = (int)min<int64_t>(rb - kb0, 32);  // first row past the boundary
        double* const vbase = V + (size_t)(cb * rstride + roff + kb0) * ldv + r0 + wn * (BN / 2) + (lane & 31);
        const int64_t jump = (rstride - rb) * ldv;
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int row = (reg & 3) + 8 * (reg >> 2) + lrow;
            if (row >= nrow) continue;
            double* vrow = vbase + (size_t)row * ldv + (row >= wrap_row ? jump : 0);
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                if (r0 + wn * (BN / 2) + tn * 32 + (lane & 31) < d) {
                    const double v = fma((double)p1[ta][tn][reg], 65536.0, (double)p2[ta][tn][reg] * 256.0) +
                                     (double)p3[ta][tn][reg];
#ifdef LGS_DIAG_BZ_NOSTORE  // diagnostic builds only: store cost probe
                    if (v == 0.5)
#endif
                    __builtin_nontemporal_store(v, vrow + tn * 32);  // streamed out, not re-read
                }
            }
        }
    } else {
        const unsigned int ukb0 = (unsigned int)kb0, urb = (unsigned int)rb;
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int row = (reg & 3) + 8 * (reg >> 2) + lrow;
            if (row >= nrow) continue;
            const unsigned int kk = ukb0 + (unsigned int)row;
            const unsigned int wrap = kk / urb;
            const int64_t orow = (cb + wrap) * rstride + roff + (kk - wrap * urb);
            double* vrow = V + (size_t)orow * ldv;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int r = r0 + wn * (BN / 2) + tn * 32 + (lane & 31);
                if (r < d) {
                    const double v = fma((double)p1[ta][tn][reg], 65536.0, (double)p2[ta][tn][reg] * 256.0) +
                                     (double)p3[ta][tn][reg];
                    __builtin_nontemporal_store(v, vrow + r);
                }
            }
        }
    }
    }
    }
    if (zmax > (ZT)32639 || zmin < (ZT)-32639) atomicOr(flags, kFlagI8Range);
}

// Moments of the kept states from bz_i8_kernel's partials: column sums over the tiles
// of the packed words, unpacked per word (the low 24 bits less the 64-row bias: sum z;
// the rest: sum z^2), exact in int64; the tile's live-chunk words (MPL) mark the
// chunks it skipped (no word written).  Skipped when the digit-range flag is up (a
// carried |z| beyond two digits: the gated moments pass recomputes them then).
__global__ __launch_bounds__(256) void bz_moments_reduce_kernel(const unsigned long long* __restrict__ MP,
                                                                const unsigned int* __restrict__ MPL,
                                                                int64_t ntiles, int64_t mp_ld, int d,
                                                                int64_t per, unsigned long long* mom,
                                                                const unsigned int* flags,
                                                                const unsigned int* abort) {
    if (aborted(abort) || (flags && (*(const volatile unsigned int*)flags & kFlagI8Range))) return;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= d) return;
    const int64_t t0 = (int64_t)blockIdx.y * per, t1 = min<int64_t>(t0 + per, ntiles);
    const int ngw = (d + 2047) / 2048;
    long long s1 = 0, s2 = 0;
    for (int64_t t = t0; t < t1; ++t) {
        if (!((MPL[(size_t)t * ngw + (i >> 11)] >> ((i >> 6) & 31)) & 1u)) continue;  // chunk all-zero in the tile
        const unsigned long long w = MP[(size_t)t * mp_ld + i];
        s1 += (long long)(w & 0xffffffull) - 64ll * 32768ll;
        s2 += (long long)(w >> 24);
    }
    atomicAdd(mom + i, (unsigned long long)s1);
    atomicAdd(mom + d + i, (unsigned long long)s2);
}

// The chains' states after a block, from the int16 history (z + 128, 16 coordinates
// of a proposal in 32 contiguous bytes) instead of the coordinate-major store (one
// 2-byte element per 64-byte line there).  Thread per (chain, 16-coordinate block),
// chain fastest.
template <typename OT>
__global__ __launch_bounds__(256) void final_h16_kernel(const int16_t* __restrict__ h16, int64_t lanes,
                                                        const int64_t* __restrict__ fsel, int64_t nc, int d,
                                                        OT* __restrict__ zs, int zs_cm,
                                                        const unsigned int* abort) {
    if (aborted(abort)) return;
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= nc) return;
    const int64_t p = fsel[c];
    if (p < 0) return;  // no proposal accepted in the block: the carried state stays
    const int b = blockIdx.y;
    const v4u_t* hp = (const v4u_t*)(h16 + ((size_t)b * lanes + p) * 16);
    const v4u_t y0 = hp[0], y1 = hp[1];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int i = 16 * b + j;
        if (i >= d) break;
        const unsigned int wv = j < 8 ? y0[j >> 1] : y1[(j - 8) >> 1];
        const OT z = (OT)((int)(short)(wv >> (16 * (j & 1))) - 128);
        if (zs_cm)
            zs[(size_t)i * nc + c] = z;
        else
            zs[(size_t)c * d + i] = z;
    }
}

// Coefficient k of each kept state (a scalar functional for lag sums):
// out[(q / rb) * rstride + roff + q % rb] = z_k of selection q (sel[q] >= 0: column
// of the proposal store, else the chain's carried-in state) -- gather_z for one row.
template <typename ZT, typename OT>
__global__ __launch_bounds__(256) void coord_gather_kernel(const ZT* __restrict__ Z, int64_t ldz,
                                                           const int64_t* __restrict__ sel, int64_t nq,
                                                           int64_t q_per_chain, const OT* __restrict__ zs,
                                                           int zs_coord_major, int64_t nc, int d, int k,
                                                           int64_t* __restrict__ out, int64_t rb, int64_t rstride,
                                                           int64_t roff, const unsigned int* abort) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq || aborted(abort)) return;
    const int64_t s = sel[q];
    int64_t v;
    if (s >= 0) {
        v = (int64_t)Z[(size_t)k * ldz + s];
    } else {
        const int64_t c = q / q_per_chain;
        v = (int64_t)(zs_coord_major ? zs[(size_t)k * nc + c] : zs[(size_t)c * d + k]);
    }
    out[(q / rb) * rstride + roff + q % rb] = v;
}

// ||v||^2 of rows q from bz_i8_kernel's partial sums VNP[k n + q], k < nparts (fixed
// order), to VN[(q / rb) * rstride + roff + q % rb].
__global__ __launch_bounds__(256) void vnorm2_reduce_kernel(const double* __restrict__ VNP, int nparts, int64_t n,
                                                            int64_t rb, int64_t rstride, int64_t roff,
                                                            double* __restrict__ VN, const unsigned int* abort) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n || aborted(abort)) return;
    double s = 0.0;
    for (int k = 0; k < nparts; ++k) s += VNP[(size_t)k * n + q];
    VN[(q / rb) * rstride + roff + q % rb] = s;
}

// Lag-L sums of per-chain scalar series continued across calls (the
// StreamingShard's LagSums, lgs_amd/distributed.py): for chains c < nc, the new values
// x[c][t] = scale * X[c ldx + t] (t < T; int64 series unscaled) after the ring's last L
// values r[c][0..L-1]: P[k nc + c] = sum_t x_t x_{t-k} for k <= L (values before the
// ring's start are 0) and P[(L + 1) nc + c] = sum_t x_t, one thread per (k, chain);
// lag_finish_kernel adds the partials to sums[k] in a fixed order and moves each ring
// to the chain's last L values.  int64 series: exact; fp64: reproducible.
template <typename T>
__device__ __forceinline__ T lag_val(const T* __restrict__ rr, const T* __restrict__ xr, int L, int64_t u,
                                     double scale) {
    if (u < L) return rr[u];  // u in [0, L + T): the ring, then the new values
    if constexpr (std::is_floating_point<T>::value) return xr[u - L] * scale;
    return xr[u - L];
}

template <typename T>
__global__ __launch_bounds__(256) void lag_partial_kernel(const T* __restrict__ X, int64_t ldx, int64_t nc,
                                                          int64_t Tn, int L, double scale,
                                                          const T* __restrict__ ring, T* __restrict__ P,
                                                          const unsigned int* abort) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t k = idx / nc, c = idx - k * nc;
    if (k > L + 1 || aborted(abort)) return;
    const T* __restrict__ xr = X + (size_t)c * ldx;
    const T* __restrict__ rr = ring + (size_t)c * L;
    T s = 0;
    if (k == L + 1) {
#pragma unroll 8
        for (int64_t t = 0; t < Tn; ++t) s += lag_val(rr, xr, L, L + t, scale);
    } else {
#pragma unroll 8
        for (int64_t t = 0; t < Tn; ++t) s += lag_val(rr, xr, L, L + t, scale) * lag_val(rr, xr, L, L + t - k, scale);
    }
    P[(size_t)k * nc + c] = s;
}

template <typename T>
__global__ __launch_bounds__(256) void lag_finish_kernel(const T* __restrict__ X, int64_t ldx, int64_t nc,
                                                         int64_t Tn, int L, double scale, T* __restrict__ ring,
                                                         const T* __restrict__ P, T* __restrict__ sums,
                                                         const unsigned int* abort) {
    if (aborted(abort)) return;
    if ((int)blockIdx.x >= L + 2) {  // ring update: ascending j reads index j + T > j, not yet written
        const int64_t c = (int64_t)(blockIdx.x - (L + 2)) * blockDim.x + threadIdx.x;
        if (c >= nc) return;
        const T* __restrict__ xr = X + (size_t)c * ldx;
        T* __restrict__ rr = ring + (size_t)c * L;
        for (int j = 0; j < L; ++j) rr[j] = lag_val(rr, xr, L, j + Tn, scale);
        return;
    }
    const int k = blockIdx.x;
    T s = 0;
    for (int64_t c = threadIdx.x; c < nc; c += 256) s += P[(size_t)k * nc + c];
    __shared__ T red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) sums[k] += red[0];
}

// ||v||^2 of rows (q / rb) * rstride + roff + q % rb of V (ld d), one wave per row,
// written (not added) to VN at the same row index: the fp64 B z paths (the int8 path
// sums them in its epilogue).  Integral v: exact in any order.
__global__ __launch_bounds__(256) void vnorm2_rows_kernel(const double* __restrict__ V, int d, int64_t n,
                                                          int64_t rb, int64_t rstride, int64_t roff,
                                                          double* __restrict__ VN, const unsigned int* abort,
                                                          const unsigned int* need) {
    const int lane = threadIdx.x & 63;
    if (aborted(abort) || not_needed(need)) return;
    // rows strided over the grid (the gated replay launches a small one)
    for (int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); q < n; q += (int64_t)gridDim.x * 4) {
        const int64_t row = (q / rb) * rstride + roff + q % rb;
        const double* __restrict__ vr = V + (size_t)row * d;
        double acc = 0.0;
        for (int j = lane; j < d; j += 64) acc = fma(vr[j], vr[j], acc);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
        if (lane == 0) VN[row] = acc;
    }
}

// ============================================================ launchers
namespace launch {

// element type dispatch on the coefficient width in bytes (2, 4, 8)
#define LGS_ZT(zb, T, ...)                 \
    do {                                   \
        if ((zb) == 2) {                   \
            using T = int16_t;             \
            __VA_ARGS__;                   \
        } else if ((zb) == 4) {            \
            using T = int32_t;             \
            __VA_ARGS__;                   \
        } else {                           \
            using T = int64_t;             \
            __VA_ARGS__;                   \
        }                                  \
    } while (0)

template <typename ZT, int PB>
static void klein_pb(const KleinArgs& a, const double* RP, const double* RC, int kernel, bool wl,
                     ZT* z, dim3 grid, hipStream_t st) {
    if (kernel == kKernelMfma) {
        const bool libm = a.szc == nullptr;
        if (PB == 32 && a.rd) {  // int8-digit far field
            if (libm && wl)
                hipLaunchKernelGGL((klein_mfma_kernel<ZT, PB, true, true, true>), grid, dim3(256), 0, st, a, RP, RC, z);
            else if (libm)
                hipLaunchKernelGGL((klein_mfma_kernel<ZT, PB, false, true, true>), grid, dim3(256), 0, st, a, RP, RC, z);
            else if (wl)
                hipLaunchKernelGGL((klein_mfma_kernel<ZT, PB, true, true>), grid, dim3(256), 0, st, a, RP, RC, z);
            else
                hipLaunchKernelGGL((klein_mfma_kernel<ZT, PB, false, true>), grid, dim3(256), 0, st, a, RP, RC, z);
        } else if (libm && wl)
            hipLaunchKernelGGL((klein_mfma_kernel<ZT, PB, true, false, true>), grid, dim3(256), 0, st, a, RP, RC, z);
        else if (libm)
            hipLaunchKernelGGL((klein_mfma_kernel<ZT, PB, false, false, true>), grid, dim3(256), 0, st, a, RP, RC, z);
        else if (wl)
            hipLaunchKernelGGL((klein_mfma_kernel<ZT, PB, true>), grid, dim3(256), 0, st, a, RP, RC, z);
        else
            hipLaunchKernelGGL((klein_mfma_kernel<ZT, PB, false>), grid, dim3(256), 0, st, a, RP, RC, z);
    } else {
        if (wl)
            hipLaunchKernelGGL((klein_panel_kernel<ZT, PB, true>), grid, dim3(256), 0, st, a, RP, RC, z);
        else
            hipLaunchKernelGGL((klein_panel_kernel<ZT, PB, false>), grid, dim3(256), 0, st, a, RP, RC, z);
    }
}

hipError_t klein(const KleinArgs& a, const double* R, const double* RP, const double* RC,
                 int panel, int kernel, bool wl, int zb, void* Z, hipStream_t st) {
    if (a.n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((a.n + 255) / 256));
    LGS_ZT(zb, ZT, {
        ZT* z = (ZT*)Z;
        if (kernel == kKernelExact) {
            if (wl)
                hipLaunchKernelGGL((klein_exact_kernel<ZT, true>), grid, dim3(256), 0, st, a, R, z);
            else
                hipLaunchKernelGGL((klein_exact_kernel<ZT, false>), grid, dim3(256), 0, st, a, R, z);
        } else if (panel == 32) {
            klein_pb<ZT, 32>(a, RP, RC, kernel, wl, z, grid, st);
        } else {
            klein_pb<ZT, 16>(a, RP, RC, kernel, wl, z, grid, st);
        }
    });
    return hipGetLastError();
}

hipError_t log_density(const KleinArgs& a, const double* R, const void* Z, int zb, double* out,
                       hipStream_t st) {
    if (a.n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((a.n + 255) / 256));
    LGS_ZT(zb, ZT, hipLaunchKernelGGL(log_density_kernel<ZT>, grid, dim3(256), 0, st, a, R, (const ZT*)Z, out));
    return hipGetLastError();
}

hipError_t samplez_probe(const double* mu, const double* sig, const double* u, int64_t n,
                         int precision, int linear, int mode, const double* etab, int64_t* z, double* ln,
                         hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(samplez_probe_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       mu, sig, u, n, precision, linear, mode, etab, z, ln);
    return hipGetLastError();
}

hipError_t accept(const AcceptArgs& a, const KleinArgs& ka, hipStream_t st) {
    if (a.nc <= 0) return hipSuccess;
    if (a.LWE)
        hipLaunchKernelGGL(imhk_accept_cert_kernel, dim3((unsigned)((a.nc + 63) / 64)), dim3(64), 0, st, a, ka);
    else
        hipLaunchKernelGGL(imhk_accept_kernel, dim3((unsigned)((a.nc + 255) / 256)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t moments_final(const void* Z, int zb, int64_t ldz, const int32_t* cnt, int64_t n, int64_t T,
                         const int64_t* fsel, int d, unsigned long long* mom, void* zs, int ob,
                         int zs_cm, int64_t nc, hipStream_t st, const unsigned int* abort,
                         const uint8_t* znz, int64_t zlanes, int zshift, const unsigned int* need) {
    if (n <= 0) return hipSuccess;
    if (zb != 2 || zlanes % 8 != 0) znz = nullptr;  // (8 proposals per flag load, 16-bit store only)
#ifdef LGS_MOM_NO_ZNZ
    znz = nullptr;
#endif
    const int64_t chunk = 16384;  // multiple of 4
#ifndef LGS_MOM_RY
#define LGS_MOM_RY 4
#endif
    constexpr int RY = LGS_MOM_RY;  // rows per workgroup, vector path
    dim3 grid((unsigned)((n + chunk - 1) / chunk), (unsigned)d);
    dim3 gridv((unsigned)((n + chunk - 1) / chunk), (unsigned)((d + RY - 1) / RY));
    if (need) {  // gated fallback: a small grid that returns at once unless needed
        grid.x = gridv.x = std::min(grid.x, 4u);
        grid.y = std::min(grid.y, 4u);
        gridv.y = std::min(gridv.y, 4u);
    }
    const int vw = zb == 2 ? 8 : 4;  // proposals per lane of the vector path
    const bool vec = ldz % vw == 0 && n % vw == 0 && ((uintptr_t)Z % (vw * (uintptr_t)zb)) == 0 &&
                     (!cnt || ((uintptr_t)cnt % 16) == 0);
    LGS_ZT(zb, ZT, LGS_ZT(ob, OT, {
        if (vec && need)
            hipLaunchKernelGGL((moments_final_kernel<ZT, OT, true, RY, true>), gridv, dim3(256), 0, st, (const ZT*)Z, ldz, cnt, n, T, fsel, d, chunk, mom, (OT*)zs, zs_cm, nc, abort, znz, zlanes, zshift, need);
        else if (vec)
            hipLaunchKernelGGL((moments_final_kernel<ZT, OT, true, RY>), gridv, dim3(256), 0, st, (const ZT*)Z, ldz, cnt, n, T, fsel, d, chunk, mom, (OT*)zs, zs_cm, nc, abort, znz, zlanes, zshift, need);
        else if (need)
            hipLaunchKernelGGL((moments_final_kernel<ZT, OT, false, 1, true>), grid, dim3(256), 0, st, (const ZT*)Z, ldz, cnt, n, T, fsel, d, chunk, mom, (OT*)zs, zs_cm, nc, abort, (const uint8_t*)nullptr, (int64_t)0, 0, need);
        else
            hipLaunchKernelGGL((moments_final_kernel<ZT, OT, false>), grid, dim3(256), 0, st, (const ZT*)Z, ldz, cnt, n, T, fsel, d, chunk, mom, (OT*)zs, zs_cm, nc, abort, (const uint8_t*)nullptr, (int64_t)0, 0, need);
    }));
    return hipGetLastError();
}

hipError_t moments_carry(const void* zs, int zb, int coord_major, int64_t nc, int d,
                         const int32_t* cc, unsigned long long* mom, hipStream_t st,
                         const unsigned int* abort, const unsigned int* need) {
    if (nc <= 0) return hipSuccess;
    const unsigned gx = need ? (unsigned)std::min(d, 16) : (unsigned)d;  // (gated: small grid)
    LGS_ZT(zb, ZT, hipLaunchKernelGGL(moments_carry_kernel<ZT>, dim3(gx), dim3(256), 0, st, (const ZT*)zs, coord_major, nc, d, cc, mom, abort, need));
    return hipGetLastError();
}

hipError_t gather_z(const void* Z, int zb, int64_t ldz, const int64_t* sel, int64_t nq,
                    int64_t q_per_chain, const void* zs, int ob, int zs_coord_major, int64_t nc,
                    int d, void* out, int out_coord_major, hipStream_t st, const unsigned int* abort) {
    if (nq <= 0) return hipSuccess;
    const dim3 grid((unsigned)((nq + 255) / 256), (unsigned)d);
    LGS_ZT(zb, ZT, LGS_ZT(ob, OT, hipLaunchKernelGGL((gather_z_kernel<ZT, OT>), grid, dim3(256), 0, st, (const ZT*)Z, ldz, sel, nq, q_per_chain, (const OT*)zs, zs_coord_major, nc, d, (OT*)out, out_coord_major, abort)));
    return hipGetLastError();
}

hipError_t lag_update(const void* X, int is_f64, int64_t ldx, int64_t nc, int64_t Tn, int L, double scale,
                      void* ring, void* sums, void* P, hipStream_t st, const unsigned int* abort) {
    if (nc <= 0 || Tn <= 0 || L < 0) return hipSuccess;
    const dim3 g1((unsigned)((nc * (L + 2) + 255) / 256)), g2((unsigned)(L + 2 + (nc + 255) / 256));
    if (is_f64) {
        hipLaunchKernelGGL(lag_partial_kernel<double>, g1, dim3(256), 0, st, (const double*)X, ldx, nc, Tn, L, scale,
                           (const double*)ring, (double*)P, abort);
        hipLaunchKernelGGL(lag_finish_kernel<double>, g2, dim3(256), 0, st, (const double*)X, ldx, nc, Tn, L, scale,
                           (double*)ring, (const double*)P, (double*)sums, abort);
    } else {
        hipLaunchKernelGGL(lag_partial_kernel<int64_t>, g1, dim3(256), 0, st, (const int64_t*)X, ldx, nc, Tn, L,
                           scale, (const int64_t*)ring, (int64_t*)P, abort);
        hipLaunchKernelGGL(lag_finish_kernel<int64_t>, g2, dim3(256), 0, st, (const int64_t*)X, ldx, nc, Tn, L,
                           scale, (int64_t*)ring, (const int64_t*)P, (int64_t*)sums, abort);
    }
    return hipGetLastError();
}

hipError_t coord_gather(const void* Z, int zb, int64_t ldz, const int64_t* sel, int64_t nq, int64_t q_per_chain,
                        const void* zs, int ob, int zs_coord_major, int64_t nc, int d, int k, int64_t* out,
                        int64_t rb, int64_t rstride, int64_t roff, hipStream_t st, const unsigned int* abort) {
    if (nq <= 0) return hipSuccess;
    LGS_ZT(zb, ZT, LGS_ZT(ob, OT, hipLaunchKernelGGL((coord_gather_kernel<ZT, OT>), dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, (const ZT*)Z, ldz, sel, nq, q_per_chain, (const OT*)zs, zs_coord_major, nc, d, k, out, rb, rstride, roff, abort)));
    return hipGetLastError();
}

hipError_t vnorm2_reduce(const double* VNP, int d, int64_t n, int64_t rb, int64_t rstride, int64_t roff,
                         double* VN, hipStream_t st, const unsigned int* abort) {
    if (n <= 0) return hipSuccess;
    const int nparts = 2 * ((d + kBzBN - 1) / kBzBN);
    hipLaunchKernelGGL(vnorm2_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, VNP, nparts, n, rb,
                       rstride, roff, VN, abort);
    return hipGetLastError();
}

hipError_t vnorm2_rows(const double* V, int d, int64_t n, int64_t rb, int64_t rstride, int64_t roff, double* VN,
                       hipStream_t st, const unsigned int* abort, const unsigned int* need) {
    if (n <= 0) return hipSuccess;
    const int64_t nb = (n + 3) / 4;
    hipLaunchKernelGGL(vnorm2_rows_kernel, dim3((unsigned)(need ? std::min<int64_t>(nb, 16) : nb)), dim3(256), 0, st,
                       V, d, n, rb, rstride, roff, VN, abort, need);
    return hipGetLastError();
}

hipError_t uninit_scan(const int32_t* init, int64_t nc, unsigned int* any, hipStream_t st) {
    if (nc <= 0) return hipSuccess;
    const unsigned g = (unsigned)std::min<int64_t>((nc + 255) / 256, 1024);
    hipLaunchKernelGGL(uninit_scan_kernel, dim3(g), dim3(256), 0, st, init, nc, any);
    return hipGetLastError();
}

hipError_t init_apply(const void* Z, int zb, int32_t* init, int64_t nc, int d, const double* LW, void* zs,
                      int ob, int zs_cm, double* lws, unsigned int* flags, hipStream_t st) {
    if (nc <= 0) return hipSuccess;
    const dim3 grid((unsigned)((nc + 255) / 256));
    LGS_ZT(zb, ZT, LGS_ZT(ob, OT, hipLaunchKernelGGL((init_apply_kernel<ZT, OT>), grid, dim3(256), 0, st, (const ZT*)Z, init, nc, d, LW, (OT*)zs, zs_cm, lws, flags)));
    return hipGetLastError();
}

hipError_t check_range16(const void* zs, int ob, int64_t count, unsigned int* flags, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    const dim3 grid((unsigned)std::min<int64_t>((count + 255) / 256, 2048));
    LGS_ZT(ob, OT, hipLaunchKernelGGL(range16_kernel<OT>, grid, dim3(256), 0, st, (const OT*)zs, count, flags));
    return hipGetLastError();
}

hipError_t carry_cols(const void* zs, int ob, int zs_coord_major, int64_t nc, int d, void* Z, int zb,
                      int64_t ldz, int64_t col0, hipStream_t st, unsigned int* flags) {
    if (nc <= 0) return hipSuccess;
    const dim3 grid((unsigned)((nc + 255) / 256), (unsigned)d);
    LGS_ZT(ob, OT, LGS_ZT(zb, ZT, hipLaunchKernelGGL((carry_cols_kernel<OT, ZT>), grid, dim3(256), 0, st, (const OT*)zs, zs_coord_major, nc, d, (ZT*)Z, ldz, col0, flags)));
    return hipGetLastError();
}

hipError_t transpose_out(const void* Z, int zb, int64_t ldz, int64_t n, int d, void* out, int ob,
                         hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 63) / 64), (unsigned)((d + 63) / 64));
    LGS_ZT(zb, ZT, LGS_ZT(ob, OT, hipLaunchKernelGGL((transpose_kernel<ZT, OT>), grid, dim3(256), 0, st, (const ZT*)Z, ldz, n, d, (OT*)out)));
    return hipGetLastError();
}

hipError_t to_coord_major(const void* in, int ib, int64_t n, int d, void* Z, int zb, int64_t ldz,
                          hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 63) / 64), (unsigned)((d + 63) / 64));
    LGS_ZT(zb, ZT, LGS_ZT(ib, IT, hipLaunchKernelGGL((to_coord_major_kernel<ZT, IT>), grid, dim3(256), 0, st, (const IT*)in, n, d, (ZT*)Z, ldz)));
    return hipGetLastError();
}

hipError_t bz(const void* Z, int zb, int64_t ldz, const int64_t* sel, const double* BT, int d,
              int64_t n, double* V, int64_t ldv, int64_t rb, int64_t rstride, int64_t roff,
              hipStream_t st, const unsigned int* abort, const unsigned int* need) {
    if (n <= 0) return hipSuccess;
    const int64_t nbx = (n + 63) / 64;  // (gated replay: 4 x 4 workgroups, each loops)
    const dim3 grid((unsigned)(need ? std::min<int64_t>(nbx, 4) : nbx),
                    (unsigned)(need ? std::min(4, (d + 63) / 64) : (d + 63) / 64));
    LGS_ZT(zb, ZT, hipLaunchKernelGGL(bz_gemm_kernel<ZT>, grid, dim3(256), 0, st, (const ZT*)Z, ldz, sel, BT, d, n, V, ldv, rb, rstride, roff, abort, need));
    return hipGetLastError();
}

hipError_t gemm_f64(const double* X, int64_t ldx, const double* MT, int d, int64_t n, double* V,
                    hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 63) / 64), (unsigned)((d + 63) / 64));
    hipLaunchKernelGGL(bz_gemm_kernel<double>, grid, dim3(256), 0, st, X, ldx, nullptr, MT, d, n, V,
                       (int64_t)d, n, (int64_t)0, (int64_t)0, (const unsigned int*)nullptr, (const unsigned int*)nullptr);
    return hipGetLastError();
}

hipError_t nearest_plane(int d, int64_t n, int panel, const double* RP, const double* RC,
                         const double* rii, const double* CP, int64_t ldc, int zb, void* Z, int64_t ldz,
                         unsigned int* flags, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 255) / 256));
    if (panel == 16)
        LGS_ZT(zb, ZT, hipLaunchKernelGGL((nearest_plane_kernel<ZT, 16>), grid, dim3(256), 0, st, d, n, RP, RC, rii, CP, ldc, (ZT*)Z, ldz, flags));
    else
        LGS_ZT(zb, ZT, hipLaunchKernelGGL((nearest_plane_kernel<ZT, 32>), grid, dim3(256), 0, st, d, n, RP, RC, rii, CP, ldc, (ZT*)Z, ldz, flags));
    return hipGetLastError();
}

hipError_t round_coeffs(const double* W, int64_t ldw, int d, int64_t n, int zb, void* Z, int64_t ldz,
                        unsigned int* flags, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 255) / 256), (unsigned)d);
    LGS_ZT(zb, ZT, hipLaunchKernelGGL(round_kernel<ZT>, grid, dim3(256), 0, st, W, ldw, d, n, (ZT*)Z, ldz, flags));
    return hipGetLastError();
}

hipError_t bz_i8(const void* Z, int zb, int64_t ldz, const int64_t* sel, const int* kchunk,
                 const int* koff, const int8_t* Bd1, const int8_t* Bd0, int dc, int d, int64_t n,
                 double* V, int64_t ldv, int64_t rb, int64_t rstride, int64_t roff,
                 unsigned int* flags, const int16_t* h16, int64_t h16_lanes, int64_t hcols,
                 hipStream_t st, const unsigned int* abort, const uint8_t* znz, const unsigned int* clive,
                 int64_t clive_ld, double* VNP, int64_t vn_n, unsigned long long* MP, int64_t mp_ld,
                 unsigned int* MPL) {
    if (n <= 0) return hipSuccess;
    if (vn_n <= 0) VNP = nullptr;
    if (d % 16 != 0 || LGS_BZ_TA != 1 || d > kOzMaxD) h16 = nullptr;  // history blocks must align with the chunks
#ifdef LGS_BZ_NO_ZNZ
    znz = nullptr;
#endif
    if (h16 == nullptr) znz = nullptr;
    if (h16 == nullptr) clive = nullptr;
#ifdef LGS_BZ_NO_CLIVE
    clive = nullptr;
#endif
    // the moment partials (MP / MPL) are written on the clive path only: never hand
    // bz_moments_reduce partials this launch will not write
    if (MP != nullptr && (clive == nullptr || !bz_moments_supported())) return hipErrorInvalidValue;
#ifdef LGS_DIAG_BZ_NO_VNP  // diagnostic builds only: epilogue cost of the ||v||^2 partial sums
    VNP = nullptr;
#endif
#ifdef LGS_DIAG_BZ_NO_SEL  // diagnostic builds only (identity selections, e.g. acceptance 1): gather cost
    sel = nullptr;
#endif
    const int tx = ((d + kBzBN - 1) / kBzBN + LGS_BZ_TXPER - 1) / LGS_BZ_TXPER;  // coordinate-tile groups
    const int64_t ty = (n + 64 * LGS_BZ_TA - 1) / (64 * LGS_BZ_TA);
    const dim3 grid((unsigned)(tx * ((ty + 7) / 8) * 8));  // whole rounds of 8 XCDs (extra tiles exit)
    LGS_ZT(zb, ZT, hipLaunchKernelGGL(bz_i8_kernel<ZT>, grid, dim3(256), 0, st, (const ZT*)Z, ldz, sel, kchunk, koff, Bd1, Bd0, dc, d, n, V, ldv, rb, rstride, roff, flags, tx, ty, h16, h16_lanes, hcols, abort, znz, clive, clive_ld, VNP, vn_n, MP, mp_ld, MPL));
    return hipGetLastError();
}

hipError_t bz_moments_reduce(const unsigned long long* MP, const unsigned int* MPL, int64_t ntiles, int64_t mp_ld,
                             int d, unsigned long long* mom, const unsigned int* flags, hipStream_t st,
                             const unsigned int* abort) {
    if (ntiles <= 0) return hipSuccess;
    const int64_t per = 32;  // tiles per workgroup
    const dim3 grid((unsigned)((d + 255) / 256), (unsigned)((ntiles + per - 1) / per));
    hipLaunchKernelGGL(bz_moments_reduce_kernel, grid, dim3(256), 0, st, MP, MPL, ntiles, mp_ld, d, per, mom,
                       flags, abort);
    return hipGetLastError();
}

hipError_t final_h16(const int16_t* h16, int64_t lanes, const int64_t* fsel, int64_t nc, int d, void* zs,
                     int ob, int zs_cm, hipStream_t st, const unsigned int* abort) {
    if (nc <= 0) return hipSuccess;
    const dim3 grid((unsigned)((nc + 255) / 256), (unsigned)((d + 15) / 16));
    LGS_ZT(ob, OT, hipLaunchKernelGGL(final_h16_kernel<OT>, grid, dim3(256), 0, st, h16, lanes, fsel, nc, d,
                                      (OT*)zs, zs_cm, abort));
    return hipGetLastError();
}

}  // namespace launch
}  // namespace lgs

#ifdef LGS_DIAG_CYCLES
// Diagnostic builds only (not part of include/lgs.h): read and reset the cycle sums.
extern "C" __attribute__((visibility("default"))) int lgs_diag_cycles_read(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lgs::lgs_diag_cycles), 16 * sizeof(unsigned long long)) !=
        hipSuccess)
        return -1;
    unsigned long long zero[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(lgs::lgs_diag_cycles), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif
#ifdef LGS_DIAG_FAR
extern "C" __attribute__((visibility("default"))) int lgs_diag_far_read(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lgs::lgs_diag_far), 8 * sizeof(unsigned long long)) != hipSuccess)
        return -1;
    unsigned long long zero[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(lgs::lgs_diag_far), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif
#ifdef LGS_DIAG_CAPQ
// Diagnostic builds only: read and reset the capped-quantile counters (lgs_device.h).
extern "C" __attribute__((visibility("default"))) int lgs_diag_capq_read(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lgs::lgs_diag_capq), 8 * sizeof(unsigned long long)) != hipSuccess)
        return -1;
    unsigned long long zero[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(lgs::lgs_diag_capq), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif
