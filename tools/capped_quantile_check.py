"""Error bounds of the capped SampleZ kind's quantile decision (lgs_device.h
sample_z_capped, sigma >= 360, window rint(mu) +- 500):
 1. max relative error of the fp64 erfinv polynomial (kCapCoef[23..36)) over
    |v| <= 0.8485 against scipy's erfinv;
 2. with exact (mpmath, 30 digits) window sums C(k) and base = P(a) - f(a)/2,
    the distance between k and xs = xe - 1/2 - (xe - m)/(24 sigma^2), xe the exact
    quantile of (C(k) + base)/sc, at the boundaries u = C(k)/S.
usage: python tools/capped_quantile_check.py   (CPU, ~1 min)
"""
import numpy as np, mpmath as mp
from scipy.special import erfinv
cf = [0.8862269447150851, 0.23200895985592382, 0.1278390124627034, 0.07920907048159789, 0.16780265291085433,
    -0.8188084361376584, 4.787814391235978, -17.187235185827564, 42.14891487326897, -68.64189227692192,
    71.76515059941498, -43.593212219926436, 11.853485934431038]
def R(x):
    p = np.zeros_like(x)
    for c in cf[::-1]: p = p * x + c
    return p
v = np.linspace(1e-12, 0.8485, 2_000_001)
rel = np.abs(v * R(v * v) - erfinv(v)) / erfinv(v)
print("erfinv poly max rel err", rel.max(), "at", v[rel.argmax()])
mp.mp.dps = 30
worst = 0
for sig in [360, 361.7, 400, 700, 1000, 5000, 1e5, 1e6, 1e10]:
    for m in [-0.5, -0.37, -0.1, 0.0, 0.23, 0.4999]:
        s = mp.mpf(sig); mm = mp.mpf(m)
        f = [mp.e ** (-(j - mm) ** 2 / (2 * s * s)) for j in range(-500, 501)]
        C = []; acc = mp.mpf(0)
        for x in f: acc += x; C.append(acc)
        # base = P(a) - f(a)/2 with exact P = s sqrt(pi/2) erf(t/sqrt2) - f * EM res  (as em_P_ld)
        t = (-500 - mm) / s
        fa = mp.e ** (-t * t / 2)
        cm = [mp.mpf(1)/12, -mp.mpf(1)/720, mp.mpf(1)/30240, -mp.mpf(1)/1209600, mp.mpf(1)/47900160, -mp.mpf(691)/1307674368000]
        hm, h, p, res, n = mp.mpf(1), t, 1 / s, mp.mpf(0), 1
        for k in range(6):
            res += cm[k] * p * h
            for r in range(2):
                h2 = t * h - n * hm; n += 1; hm = h; h = h2
            p /= s * s
        PA = s * mp.sqrt(mp.pi / 2) * mp.erf(t / mp.sqrt(2)) - fa * res
        base = PA - fa / 2
        sc = s * mp.sqrt(mp.pi / 2)
        mx = 0
        for k in list(range(-501, 500, 7)) + [-501, -500, 499, 498]:
            Ck = C[k + 500] if k >= -500 else mp.mpf(0)
            vk = (Ck + base) / sc
            xe = mm + s * mp.sqrt(2) * mp.erfinv(vk)
            xs = xe - mp.mpf(1) / 2 - (xe - mm) / (24 * s * s)
            r = abs(xs - k)
            mx = max(mx, r)
        worst = max(worst, mx)
        print(sig, m, float(mx), float(mx * 48 * sig * sig))
print("worst", float(worst))
