"""Distribution of |lw_default - lw_exact| (Wang-Ling weights) over 16384 C3 samples,
with the default SampleZ path and with LGS_SAMPLEZ_LIBM; the worst sample's z kinds."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lattice-gaussian-mcmc_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import lgs_oracle as oracle  # noqa: E402
from lgs_amd import _capi  # noqa: E402
from lgs_amd.lattices import build_config  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3_ntru512"
lat, sigma = build_config(cfg)
B = lat.basis
d = B.shape[0]
R, cp = oracle.qr_prepare(B)
ctx = _capi.Context(0)
ctx.set_basis(R, cp, B, sigma)
n = 1 << 14
base = _capi.LGS_DEVICE_PTRS | _capi.LGS_COORD_MAJOR | _capi.LGS_WANG_LING
res = {}
for name, extra in (("default", 0), ("libm", _capi.LGS_SAMPLEZ_LIBM), ("exact", _capi.LGS_EXACT_ORDER)):
    z = torch.empty((d, n), dtype=torch.int32, device="cuda")
    lw = torch.empty(n, dtype=torch.float64, device="cuda")
    ctx.klein(91, 0, n, z, None, lw, base | extra)
    torch.cuda.synchronize()
    res[name] = (z.cpu().numpy(), lw.cpu().numpy())
for name in ("default", "libm"):
    diff = np.abs(res[name][1] - res["exact"][1])
    same_z = np.array_equal(res[name][0], res["exact"][0])
    q = np.quantile(diff, [0.5, 0.99, 0.999, 1.0])
    w = int(np.argmax(diff))
    print(f"{cfg} {name}: z equal {same_z}; |dlw| median {q[0]:.2e} p99 {q[1]:.2e} p99.9 {q[2]:.2e} max {q[3]:.2e} "
          f"(sample {w}, lw {res['exact'][1][w]:.6f}); samples > 1e-6: {int((diff > 1e-6).sum())}", flush=True)
w = int(np.argmax(np.abs(res["default"][1] - res["exact"][1])))
zw = res["exact"][0][:, w]
sig_i = sigma / np.diag(R)
big = np.flatnonzero(np.abs(zw) > 0)
print(f"worst sample {w}: {big.size} nonzero coordinates; sigma_i range {sig_i.min():.3g}..{sig_i.max():.3g}; "
      f"max |z| {np.abs(zw).max()} at i={int(np.argmax(np.abs(zw)))} (sigma_i {sig_i[int(np.argmax(np.abs(zw)))]:.4g})")
ref = oracle.log_weight(R, cp, B, sigma, zw.astype(np.int64), mode=oracle.IMHK_WANG_LING)
print(f"worst sample oracle {ref:.10f} default {res['default'][1][w]:.10f} exact {res['exact'][1][w]:.10f}")
