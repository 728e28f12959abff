// lgs_szc_host.h -- host-side builder of the per-coordinate SampleZ constants
// (layout and kinds: lgs_kernels.h kSzc*), used by lgs_set_basis and by the
// SampleZ micro-benchmark.  Long-double evaluation of the Euler-Maclaurin
// window sums of lgs_device.h; see DESIGN.md §SampleZ.
#pragma once
#include <algorithm>
#include <cmath>

#include "lgs_kernels.h"

namespace lgs_host {

// ---------------------------------------------------------------- SampleZ constants
// Euler-Maclaurin antiderivative P(t) of lgs_device.h (em_P) in long double:
// P = sigma sqrt(pi/2) erf(t/sqrt2) - f(t) sum_{m<=6} c_m He_{2m-1}(t)/sigma^(2m-1).
constexpr long double kPiL = 3.141592653589793238462643383279502884L;

inline long double em_P_ld(long double t, long double sig, long double& f) {
    static const long double cm[6] = {1.0L / 12.0L, -1.0L / 720.0L, 1.0L / 30240.0L,
                                      -1.0L / 1209600.0L, 1.0L / 47900160.0L,
                                      -691.0L / 1307674368000.0L};
    f = expl(-0.5L * t * t);
    long double hm = 1.0L, h = t, p = 1.0L / sig, res = 0.0L, n = 1.0L;
    for (int m = 0; m < 6; ++m) {
        res += cm[m] * p * h;
        for (int r = 0; r < 2; ++r) {
            const long double h2 = t * h - n * hm;
            n += 1.0L;
            hm = h;
            h = h2;
        }
        p /= sig * sig;
    }
    return sig * sqrtl(kPiL / 2.0L) * erfl(t / sqrtl(2.0L)) - f * res;
}

// Window normaliser S(m) and base(m) = P(lo) - f(lo)/2 of the capped window
// [c-500, c+500], c = rint(mu), as functions of m = mu - c.
inline void capped_S_base(long double m, long double sig, long double& S, long double& base) {
    long double fL, fU;
    const long double PL = em_P_ld((-500.0L - m) / sig, sig, fL);
    const long double PU = em_P_ld((500.0L - m) / sig, sig, fU);
    S = (PU - PL) + 0.5L * (fL + fU);
    base = PL - 0.5L * fL;
}

// Fills the kSzcStride constants of one coordinate (layout: lgs_kernels.h).
inline void build_szc(double s, int precision, double* q) {
    std::fill(q, q + lgs::kSzcStride, 0.0);
    q[0] = s;
    if (s == 0.0) {
        q[2] = lgs::kSzRound;
        return;
    }
    const double kSqrtHalfPi = 1.2533141373155003, kSqrt2 = 1.4142135623730951;
    const double rf = (s < 0.1) ? (double)(precision > 3 ? precision : 3) : (double)precision;
    q[1] = 1.0 / s;
    q[3] = s * kSqrtHalfPi;
    q[4] = 1.0 / q[3];
    q[5] = s * kSqrt2;
    q[6] = rf * s;
    if (s < 4.0) {
        q[2] = lgs::kSzSmall;
        // a point entering / leaving at a window end lies >= q6 + 1 from mu while a
        // window point lies within 1/2: relative mass <= exp(-((q6+1)^2 - 1/4) / (2 s^2))
        // q[7]: 0 -- such a point's probability is exactly 0 in fp64 (e^-746); 0.5 --
        // below 2^-60 = e^-41.6 (matters only for u = 0); 1 -- the ends are checked
        const double e = ((q[6] + 1.0) * (q[6] + 1.0) - 0.25) / (2.0 * s * s);
        q[7] = e > 746.0 ? 0.0 : (e > 42.0 ? 0.5 : 1.0);
        return;
    }
    const double W = 2.0 * q[6];
    if (W + 2.0 <= 1000.0 && precision >= 9) {
        q[2] = lgs::kSzClosed;
        q[7] = q[3] + q[3];
        q[8] = -q[3];
        return;
    }
    q[2] = lgs::kSzGeneric;
    if (!(W > 1000.0)) return;
    // Chebyshev interpolation on m in [-1/2, 1/2] (x = 2m), converted to monomials in m.
    const int N = lgs::kSzDeg + 1;
    long double fs[N], fb[N], as[N], ab[N];
    const long double sg = s;
    for (int k = 0; k < N; ++k) {
        const long double x = cosl(kPiL * (k + 0.5L) / N);
        capped_S_base(0.5L * x, sg, fs[k], fb[k]);
    }
    for (int j = 0; j < N; ++j) {
        long double ss = 0, sb = 0;
        for (int k = 0; k < N; ++k) {
            const long double w = cosl(kPiL * j * (k + 0.5L) / N);
            ss += fs[k] * w;
            sb += fb[k] * w;
        }
        as[j] = ss * (j ? 2.0L : 1.0L) / N;
        ab[j] = sb * (j ? 2.0L : 1.0L) / N;
    }
    // T_j(x) -> monomials in x (recurrence), then x = 2m.
    long double Tm[N][N] = {};
    Tm[0][0] = 1.0L;
    if (N > 1) Tm[1][1] = 1.0L;
    for (int j = 2; j < N; ++j)
        for (int k = 0; k < N; ++k)
            Tm[j][k] = (k ? 2.0L * Tm[j - 1][k - 1] : 0.0L) - Tm[j - 2][k];
    long double cs[N] = {}, cb[N] = {};
    for (int j = 0; j < N; ++j)
        for (int k = 0; k < N; ++k) {
            cs[k] += as[j] * Tm[j][k];
            cb[k] += ab[j] * Tm[j][k];
        }
    long double scale = 1.0L;
    for (int k = 0; k < N; ++k) {
        q[lgs::kSzS + k] = (double)(cs[k] * scale);
        q[lgs::kSzB + k] = (double)(cb[k] * scale);
        scale *= 2.0L;
    }
    // check the fp64 Horner evaluation against long double at 33 points; a fit that
    // is not within ~2 ulp of S keeps the generic per-draw evaluation
    long double err = 0.0L, Smin = 1e300L;
    for (int t = 0; t <= 32; ++t) {
        const double m = -0.5 + t / 32.0;
        long double Se, be;
        capped_S_base(m, sg, Se, be);
        double S = q[lgs::kSzS + lgs::kSzDeg], b = q[lgs::kSzB + lgs::kSzDeg];
        for (int k = lgs::kSzDeg - 1; k >= 0; --k) {
            S = std::fma(S, m, q[lgs::kSzS + k]);
            b = std::fma(b, m, q[lgs::kSzB + k]);
        }
        err = std::max(err, std::max(fabsl((long double)S - Se), fabsl((long double)b - be)));
        Smin = std::min(Smin, Se);
    }
    if (err <= 5e-16L * Smin) {  // ~2 ulp of S
        q[2] = lgs::kSzCapped;
        // |k - mu| <= 500.5 in the window: |k - mu| / (sigma sqrt 2) <= 1 from sigma >=
        // 354, the range of the series erf / exp (lgs_device.h PolyErf)
        q[7] = s >= 360.0 ? 1.0 : 0.0;
    }
}

}  // namespace lgs_host
