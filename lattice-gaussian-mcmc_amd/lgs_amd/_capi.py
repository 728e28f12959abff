"""ctypes binding of the HIP C-ABI (``include/lgs.h`` -> ``lgs_amd/_lib/liblgs_hip.so``).

This is the only way the package computes anything: there is no CPU fallback.
If the library is missing, or no HIP device is visible, constructing a
``Context`` raises ``LgsError`` immediately.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LGS_LIB") or os.path.join(_HERE, "_lib", "liblgs_hip.so")
# the same sources built with -DLGS_TEST_HOOKS (the environment's test / A/B switches):
# only tests that perturb the certificate on purpose use it (Context(hooks=True))
HOOKS_LIB_PATH = os.path.join(_HERE, "_lib", "liblgs_hip_hooks.so")

LGS_OK = 0
LGS_ERR_INVALID = -1
LGS_ERR_HIP = -2
LGS_ERR_NOMEM = -3
LGS_ERR_OVERFLOW = -4
LGS_ERR_NONFINITE = -5
LGS_ERR_STATE = -6

LGS_BASIS_LINEAR_PROBS = 0x1
LGS_DEVICE_PTRS = 0x1
LGS_EXACT_ORDER = 0x2
LGS_WANG_LING = 0x4
LGS_Z64 = 0x8
LGS_COORD_MAJOR = 0x10
LGS_SAMPLEZ_TABLE = 0x20
LGS_SAMPLEZ_DECISION = 0x40
LGS_SAMPLEZ_LIBM = 0x80
LGS_LOGW_BOUND = 0x400

LGS_X_I32 = 0x100
LGS_X_I64 = 0x200

# lgs_create_ex ctx_flags (include/lgs.h)
LGS_CTX_NO_PIPELINE = 0x1
LGS_CTX_NO_LOOKAHEAD = 0x2
LGS_CTX_SAMPLEZ_LIBM = 0x4
LGS_CTX_PANEL16 = 0x8
LGS_CTX_FAR_FP64 = 0x10
LGS_CTX_STORE32 = 0x20
LGS_CTX_NO_QSKIP = 0x40
LGS_CTX_NO_CU_SPLIT = 0x80

KERNEL_KLEIN, KERNEL_BZ, KERNEL_ACCEPT, KERNEL_MOMENTS = 0, 1, 2, 3
KERNEL_GRAM, KERNEL_SERIES, KERNEL_KLEIN_INIT = 4, 5, 6
LGS_COUNTER_RESOLVED = 0
LGS_COUNTER_FALLBACK = 1
LGS_COUNTER_ACCEPT_RESOLVED = 2
LGS_COUNTER_WL_MISMATCH = 3
LGS_COUNTER_QSKIP = 4
LGS_COUNTER_KLEIN_CUS = 5

# every symbol include/lgs.h declares (checked by tests/test_capi_symbols.py)
EXPORTS = ("lgs_version", "lgs_last_error", "lgs_create", "lgs_create_ex", "lgs_destroy", "lgs_set_stream",
           "lgs_set_basis", "lgs_klein", "lgs_imhk", "lgs_imhk_trace", "lgs_imhk_ex", "lgs_lattice_points", "lgs_log_density", "lgs_sample_z", "lgs_timing_enable",
           "lgs_timing_get", "lgs_device_info", "lgs_series_stats", "lgs_gram",
           "lgs_jump_distance", "lgs_marginal_tvd", "lgs_column_range", "lgs_histogram", "lgs_set_decoder", "lgs_nearest_plane",
           "lgs_round_decode", "lgs_counter")


class ImhkOutputs(ctypes.Structure):
    """struct lgs_imhk_outputs (include/lgs.h)."""
    _fields_ = [("logw_samples", ctypes.c_void_p), ("accepted", ctypes.c_void_p),
                ("vnorm2_samples", ctypes.c_void_p), ("zk_samples", ctypes.c_void_p),
                ("zk_index", ctypes.c_int64), ("fn_chains", ctypes.c_int64),
                ("lag_L", ctypes.c_int64), ("lag_z_ring", ctypes.c_void_p), ("lag_z_sums", ctypes.c_void_p),
                ("lag_v_ring", ctypes.c_void_p), ("lag_v_sums", ctypes.c_void_p), ("lag_v_scale", ctypes.c_double)]


class LgsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"lgs error {code}: {msg}")
        self.code = code


_lib = None   # the library at LIB_PATH (the product unless LGS_LIB names a variant)
_libs = {}    # every library loaded, by path
_vp = ctypes.c_void_p
_dp = ctypes.POINTER(ctypes.c_double)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)


def load_library(path: str = LIB_PATH):
    """Load liblgs_hip.so (raises if it has not been built)."""
    global _lib
    if path in _libs:
        return _libs[path]
    # One HIP runtime per process: PyTorch ships its own libamdhip64 (soname
    # libamdhip64.so.7) and binds it by the unversioned name, so it must be
    # loaded first; liblgs_hip.so's NEEDED libamdhip64.so.7 then resolves to the
    # same runtime and device pointers / streams are shared with torch.
    if os.environ.get("LGS_NO_TORCH") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    if not os.path.exists(path):
        raise LgsError(LGS_ERR_STATE, f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(path)
    L.lgs_version.restype = ctypes.c_int
    L.lgs_last_error.restype = ctypes.c_char_p
    L.lgs_create.argtypes = [ctypes.POINTER(_vp), ctypes.c_int]
    if hasattr(L, "lgs_create_ex"):  # (round 6; older A/B baselines lack it)
        L.lgs_create_ex.argtypes = [ctypes.POINTER(_vp), ctypes.c_int, ctypes.c_int64, ctypes.c_uint32]
    L.lgs_destroy.argtypes = [_vp]
    L.lgs_set_stream.argtypes = [_vp, _vp]
    L.lgs_set_basis.argtypes = [_vp, ctypes.c_int64, _dp, _dp, _dp, ctypes.c_double, ctypes.c_int32,
                                ctypes.c_uint32]
    L.lgs_klein.argtypes = [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64, _vp, _vp, _vp,
                            ctypes.c_uint32]
    L.lgs_imhk.argtypes = [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint64,
                           ctypes.c_int64, ctypes.c_int32, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                           ctypes.c_uint32]
    L.lgs_imhk_trace.argtypes = [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint64,
                                 ctypes.c_int64, ctypes.c_int32, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                 _vp, _vp, ctypes.c_uint32]
    if hasattr(L, "lgs_imhk_ex"):  # (round 4; older builds, e.g. A/B baselines, lack it)
        L.lgs_imhk_ex.argtypes = [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint64,
                                  ctypes.c_int64, ctypes.c_int32, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                  ctypes.POINTER(ImhkOutputs), ctypes.c_uint32]
    L.lgs_lattice_points.argtypes = [_vp, ctypes.c_int64, _vp, _vp, ctypes.c_uint32]
    L.lgs_log_density.argtypes = [_vp, ctypes.c_int64, _vp, _vp, ctypes.c_uint32]
    L.lgs_sample_z.argtypes = [_vp, ctypes.c_int64, _vp, _vp, _vp, ctypes.c_int32, _vp, _vp,
                               ctypes.c_uint32]
    L.lgs_timing_enable.argtypes = [_vp, ctypes.c_int]
    L.lgs_timing_get.argtypes = [_vp, ctypes.c_int, _dp, _i64p]
    L.lgs_counter.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
    L.lgs_device_info.argtypes = [_vp, ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                  _i64p]
    _i64 = ctypes.c_int64
    L.lgs_series_stats.argtypes = [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64,
                                   ctypes.c_double, _i64, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint32]
    L.lgs_gram.argtypes = [_vp, _i64, _i64, _vp, _i64, _vp, _vp, _vp, ctypes.c_uint32]
    L.lgs_jump_distance.argtypes = [_vp, _i64, _i64, _vp, _i64, _vp, ctypes.c_uint32]
    L.lgs_marginal_tvd.argtypes = [_vp, _i64, _vp, _i64, _vp, _i64, _vp, ctypes.c_uint32]
    L.lgs_column_range.argtypes = [_vp, _i64, _vp, _i64, _vp, _vp, ctypes.c_uint32]
    L.lgs_histogram.argtypes = [_vp, _i64, _vp, _i64, _i64, _vp, _vp, _vp, ctypes.c_uint32]
    L.lgs_set_decoder.argtypes = [_vp, _vp, _vp]
    L.lgs_nearest_plane.argtypes = [_vp, _i64, _vp, _vp, _vp, ctypes.c_uint32]
    L.lgs_round_decode.argtypes = [_vp, _i64, _vp, _vp, _vp, ctypes.c_uint32]
    for name in EXPORTS:
        if name not in ("lgs_version", "lgs_last_error") and hasattr(L, name):
            getattr(L, name).restype = ctypes.c_int
    _libs[path] = L
    if path == LIB_PATH:
        _lib = L
    return L


def _check(rc, L=None):
    if rc != LGS_OK:
        msg = (L or _lib or load_library()).lgs_last_error().decode(errors="replace")
        raise LgsError(rc, msg)


def _ptr(a):
    """Host numpy array or device tensor (anything with data_ptr()) -> void*."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        if not a.flags.c_contiguous:
            raise ValueError("arrays must be C-contiguous")
        return ctypes.c_void_p(a.ctypes.data)
    if hasattr(a, "data_ptr"):
        if hasattr(a, "is_contiguous") and not a.is_contiguous():
            raise ValueError("tensors must be contiguous")
        return ctypes.c_void_p(a.data_ptr())
    if isinstance(a, int):
        return ctypes.c_void_p(a)
    raise TypeError(f"unsupported buffer {type(a)}")


def _dtype_name(a):
    return str(a.dtype).replace("torch.", "")


def _check_bufs(flags, device, bufs):
    """Caller buffers must match the call's flags: element type (LGS_Z64 selects
    int64 coefficients), and host vs device memory (LGS_DEVICE_PTRS, on the
    context's device) -- a mismatch would be silently misread by the library."""
    dev_flag = bool(flags & LGS_DEVICE_PTRS)
    for a, want, name in bufs:
        if a is None or isinstance(a, int):  # raw addresses are opaque: the caller vouches for them
            continue
        got = _dtype_name(a)
        if got != want:
            raise ValueError(f"{name}: expected {want}, got {got}")
        is_dev = bool(getattr(a, "is_cuda", False))
        if is_dev != dev_flag:
            raise ValueError(f"{name}: {'device' if is_dev else 'host'} buffer with LGS_DEVICE_PTRS "
                             f"{'set' if dev_flag else 'unset'}")
        if is_dev and a.device.index is not None and a.device.index != device:
            raise ValueError(f"{name}: on cuda:{a.device.index}, context on cuda:{device}")


def x_flags(a) -> int:
    """LGS_X_* element-type flag of a host array / device tensor (fp64, int32, int64)."""
    t = _dtype_name(a)
    if t == "float64":
        return 0
    if t == "int32":
        return LGS_X_I32
    if t == "int64":
        return LGS_X_I64
    raise TypeError(f"diagnostics take float64 / int32 / int64 data, got {t}")


class Context:
    """One HIP device context (stream + device-resident basis + scratch)."""

    def __init__(self, device: int = 0, *, max_proposals: int = 0, pipeline: bool = True,
                 lookahead: bool = True, samplez_libm: bool = False, panel: int = 32, far: str = "int8",
                 store32: bool = False, qskip: bool = True, cu_split: bool = True,
                 hooks: bool = False):
        """lgs_create_ex: max_proposals (0 = the library's default) and the LGS_CTX_*
        options; hooks=True loads liblgs_hip_hooks.so (the environment's test switches)."""
        L = load_library(HOOKS_LIB_PATH if hooks else LIB_PATH)
        self._L = L
        flags = ((0 if pipeline else LGS_CTX_NO_PIPELINE) | (0 if lookahead else LGS_CTX_NO_LOOKAHEAD) |
                 (LGS_CTX_SAMPLEZ_LIBM if samplez_libm else 0) | (LGS_CTX_PANEL16 if panel == 16 else 0) |
                 (LGS_CTX_FAR_FP64 if far == "fp64" else 0) | (LGS_CTX_STORE32 if store32 else 0) |
                 (0 if qskip else LGS_CTX_NO_QSKIP) | (0 if cu_split else LGS_CTX_NO_CU_SPLIT))
        if panel not in (16, 32) or far not in ("int8", "fp64"):
            raise ValueError("panel is 16 or 32, far is 'int8' or 'fp64'")
        h = _vp()
        if hasattr(L, "lgs_create_ex"):
            _check(L.lgs_create_ex(ctypes.byref(h), int(device), int(max_proposals), flags), L)
        elif flags or max_proposals:
            raise LgsError(LGS_ERR_INVALID, "this library build has no lgs_create_ex")
        else:
            _check(L.lgs_create(ctypes.byref(h), int(device)), L)
        self._h = h
        self.device = device
        self.d = 0

    def _ck(self, rc):
        _check(rc, self._L)

    def close(self):
        if getattr(self, "_h", None) and getattr(self, "_L", None) is not None:
            self._L.lgs_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    # ---------------------------------------------------------------- setup
    def set_stream(self, stream_handle):
        self._ck(self._L.lgs_set_stream(self._h, _vp(stream_handle) if stream_handle else None))

    def set_basis(self, R, cprime, B, sigma, precision=10, linear_probs=False):
        R = np.ascontiguousarray(R, dtype=np.float64)
        cp = np.ascontiguousarray(cprime, dtype=np.float64)
        Bc = None if B is None else np.ascontiguousarray(B, dtype=np.float64)
        d = R.shape[0]
        if R.shape != (d, d) or cp.shape != (d,) or (Bc is not None and Bc.shape != (d, d)):
            raise ValueError("shape mismatch between R, cprime and B")
        flags = LGS_BASIS_LINEAR_PROBS if linear_probs else 0
        self._ck(self._L.lgs_set_basis(self._h, d, R.ctypes.data_as(_dp), cp.ctypes.data_as(_dp),
                                  None if Bc is None else Bc.ctypes.data_as(_dp), float(sigma),
                                  int(precision), flags))
        self.d = d
        self._keep = (R, cp, Bc)

    # ---------------------------------------------------------------- compute
    def klein(self, seed, first, n, z_out=None, v_out=None, logw_out=None, flags=0):
        """Raw lgs_klein on caller-provided buffers (numpy host or device tensors)."""
        zt = "int64" if flags & LGS_Z64 else "int32"
        _check_bufs(flags, self.device, ((z_out, zt, "z_out"), (v_out, "float64", "v_out"),
                                         (logw_out, "float64", "logw_out")))
        self._ck(self._L.lgs_klein(self._h, int(seed) & 0xFFFFFFFFFFFFFFFF, int(first), int(n),
                              _ptr(z_out), _ptr(v_out), _ptr(logw_out), int(flags)))

    def klein_host(self, seed, first, n, *, want_z=True, want_v=True, want_logw=False, flags=0):
        """Klein samples into fresh host arrays; int32 first, int64 on overflow."""
        d = self.d
        for z64 in (False, True):
            f = flags | (LGS_Z64 if z64 else 0)
            z = np.empty((n, d), dtype=np.int64 if z64 else np.int32) if want_z else None
            v = np.empty((n, d)) if want_v else None
            lw = np.empty(n) if want_logw else None
            try:
                self.klein(seed, first, n, z, v, lw, f)
            except LgsError as e:
                if e.code == LGS_ERR_OVERFLOW and not z64:
                    continue
                raise
            return {"z": None if z is None else z.astype(np.int64, copy=False), "v": v, "logw": lw}
        raise AssertionError("unreachable")

    def imhk(self, seed, first_chain, n_chains, first_step, n_steps, thin, z_state, logw_state,
             state_init, accepts, z_samples=None, v_samples=None, moments=None, flags=0,
             logw_samples=None, accepted=None, vnorm2_samples=None, zk_samples=None, zk_index=0,
             fn_chains=0, lag=None):
        """lgs_imhk; with logw_samples (n_chains x n_steps/thin float64) or accepted
        (n_chains x n_steps uint8) lgs_imhk_trace, which also records each kept
        state's log weight and each step's accept decision; with vnorm2_samples /
        zk_samples (n_chains x n_steps/thin float64 / int64, device) lgs_imhk_ex, which
        also gives ||v||^2 and coefficient zk_index of each kept state (fn_chains > 0:
        of the leading fn_chains chains only, arrays fn_chains x n_steps/thin); lag =
        (L, z_ring, z_sums, v_ring, v_sums, v_scale): device buffers whose lag-0..L sums
        of both series the call continues (include/lgs.h lgs_imhk_outputs.lag_L)."""
        zt = "int64" if flags & LGS_Z64 else "int32"
        _check_bufs(flags, self.device, ((z_state, zt, "z_state"), (logw_state, "float64", "logw_state"),
                                         (state_init, "int32", "state_init"), (accepts, "int64", "accepts"),
                                         (z_samples, zt, "z_samples"), (v_samples, "float64", "v_samples"),
                                         (moments, "int64", "moments"), (logw_samples, "float64", "logw_samples"),
                                         (accepted, "uint8", "accepted")))
        args = (self._h, int(seed) & 0xFFFFFFFFFFFFFFFF, int(first_chain), int(n_chains), int(first_step),
                int(n_steps), int(thin), _ptr(z_state), _ptr(logw_state), _ptr(state_init), _ptr(accepts),
                _ptr(z_samples), _ptr(v_samples), _ptr(moments))
        if vnorm2_samples is not None or zk_samples is not None:
            _check_bufs(flags, self.device, ((vnorm2_samples, "float64", "vnorm2_samples"),
                                             (zk_samples, "int64", "zk_samples")))
            def v(a):
                q = _ptr(a)
                return None if q is None else q.value
            lg = (0, None, None, None, None, 0.0) if lag is None else lag
            if lag is not None:
                _check_bufs(flags, self.device, ((lg[1], "int64", "lag z ring"), (lg[2], "int64", "lag z sums"),
                                                 (lg[3], "float64", "lag v ring"), (lg[4], "float64", "lag v sums")))
            out = ImhkOutputs(v(logw_samples), v(accepted), v(vnorm2_samples), v(zk_samples), int(zk_index),
                              int(fn_chains), int(lg[0]), v(lg[1]), v(lg[2]), v(lg[3]), v(lg[4]), float(lg[5]))
            self._ck(self._L.lgs_imhk_ex(*args, ctypes.byref(out), int(flags)))
        elif logw_samples is None and accepted is None:
            self._ck(self._L.lgs_imhk(*args, int(flags)))
        else:
            self._ck(self._L.lgs_imhk_trace(*args, _ptr(logw_samples), _ptr(accepted), int(flags)))

    def lattice_points(self, z, v_out=None, flags=0):
        if isinstance(z, np.ndarray):
            z64 = z.dtype == np.int64
            zz = np.ascontiguousarray(z, dtype=np.int64 if z64 else np.int32)
            n = zz.shape[0]
            v = np.empty((n, self.d)) if v_out is None else v_out
            self._ck(self._L.lgs_lattice_points(self._h, n, _ptr(zz), _ptr(v),
                                           int(flags | (LGS_Z64 if z64 else 0))))
            return v
        n = z.shape[0] if not (flags & LGS_COORD_MAJOR) else z.shape[1]
        self._ck(self._L.lgs_lattice_points(self._h, n, _ptr(z), _ptr(v_out), int(flags)))
        return v_out

    def log_density(self, z):
        zz = np.ascontiguousarray(z)
        z64 = zz.dtype == np.int64
        if not z64:
            zz = zz.astype(np.int32)
        out = np.empty(zz.shape[0])
        self._ck(self._L.lgs_log_density(self._h, zz.shape[0], _ptr(zz), _ptr(out),
                                    LGS_Z64 if z64 else 0))
        return out

    def sample_z(self, mu, sigma, u, precision=10, table=False, linear_probs=False, mode=None):
        mu = np.ascontiguousarray(mu, dtype=np.float64)
        sg = np.ascontiguousarray(np.broadcast_to(sigma, mu.shape), dtype=np.float64)
        uu = np.ascontiguousarray(u, dtype=np.float64)
        z = np.empty(mu.shape, dtype=np.int64)
        ln = np.empty(mu.shape)
        f = (LGS_SAMPLEZ_TABLE if table else 0) | (LGS_BASIS_LINEAR_PROBS if linear_probs else 0)
        f |= {None: 0, "decision": LGS_SAMPLEZ_DECISION, "libm": LGS_SAMPLEZ_LIBM,
              "libm_decision": LGS_SAMPLEZ_LIBM | LGS_SAMPLEZ_DECISION}[mode]
        self._ck(self._L.lgs_sample_z(self._h, mu.size, _ptr(mu), _ptr(sg), _ptr(uu), int(precision),
                                 _ptr(z), _ptr(ln), f))
        return z, ln

    # ---------------------------------------------------------------- decoding
    def set_decoder(self, Q=None, Binv=None):
        Qc = None if Q is None else np.ascontiguousarray(Q, dtype=np.float64)
        Bi = None if Binv is None else np.ascontiguousarray(Binv, dtype=np.float64)
        for M in (Qc, Bi):
            if M is not None and M.shape != (self.d, self.d):
                raise ValueError("decoder matrices must be d x d")
        self._ck(self._L.lgs_set_decoder(self._h, _ptr(Qc), _ptr(Bi)))
        self._keep_dec = (Qc, Bi)

    def decode(self, targets, method="plane", z_out=None, v_out=None, flags=0):
        """Raw lgs_nearest_plane / lgs_round_decode on caller buffers."""
        fn = self._L.lgs_nearest_plane if method == "plane" else self._L.lgs_round_decode
        n = targets.shape[1] if flags & LGS_COORD_MAJOR else targets.shape[0]
        self._ck(fn(self._h, int(n), _ptr(targets), _ptr(z_out), _ptr(v_out), int(flags)))

    def decode_host(self, targets, method="plane", want_v=True):
        """Decode host targets (n x d); int32 coefficients first, int64 on overflow."""
        t = np.ascontiguousarray(targets, dtype=np.float64)
        n = t.shape[0]
        for z64 in (False, True):
            z = np.empty((n, self.d), dtype=np.int64 if z64 else np.int32)
            v = np.empty((n, self.d)) if want_v else None
            try:
                self.decode(t, method, z, v, LGS_Z64 if z64 else 0)
            except LgsError as e:
                if e.code == LGS_ERR_OVERFLOW and not z64:
                    continue
                raise
            return z.astype(np.int64, copy=False), v
        raise AssertionError("unreachable")

    # ---------------------------------------------------------------- diagnostics
    def series_stats(self, x, n_series, n, group_size, group_stride, series_stride, time_stride,
                     max_lag=-1, window_c=5.0, batch_size=0, mean=None, c0=None, acf=None,
                     tau=None, batch_means=None, flags=0):
        """Raw lgs_series_stats; x / outputs are host arrays or device tensors
        (flags must then carry LGS_DEVICE_PTRS); element type via x_flags(x)."""
        self._ck(self._L.lgs_series_stats(self._h, _ptr(x), int(n_series), int(n), int(group_size),
                                     int(group_stride), int(series_stride), int(time_stride),
                                     int(max_lag), float(window_c), int(batch_size), _ptr(mean),
                                     _ptr(c0), _ptr(acf), _ptr(tau), _ptr(batch_means),
                                     int(flags | x_flags(x))))

    def gram(self, x, shift=None, sum_out=None, gram_out=None, coord_major=False, flags=0):
        """sum y and sum y y^T, y = x - shift, ADDED to sum_out (d) / gram_out (d x d):
        int64 (exact) for int32 / int64 x, fp64 for float64 x."""
        f = flags | (LGS_COORD_MAJOR if coord_major else 0) | x_flags(x)
        if coord_major:
            d, n = x.shape
        else:
            n, d = x.shape
        self._ck(self._L.lgs_gram(self._h, int(d), int(n), _ptr(x), int(n if coord_major else d),
                             _ptr(shift), _ptr(sum_out), _ptr(gram_out), int(f)))

    def jump_distance(self, x, out, flags=0):
        n, d = x.shape
        self._ck(self._L.lgs_jump_distance(self._h, int(n), int(d), _ptr(x), int(d), _ptr(out),
                                      int(flags | x_flags(x))))

    def marginal_tvd(self, x1, x2, out, flags=0):
        if _dtype_name(x1) != _dtype_name(x2):
            raise TypeError("both sample sets must have the same dtype")
        d = x1.shape[1]
        self._ck(self._L.lgs_marginal_tvd(self._h, int(d), _ptr(x1), int(x1.shape[0]), _ptr(x2),
                                     int(x2.shape[0]), _ptr(out), int(flags | x_flags(x1))))

    def column_range(self, x, lo, hi, flags=0):
        """Per-column min / max (fp64) of row-major (n, d) samples into lo / hi (d)."""
        n, d = x.shape
        self._ck(self._L.lgs_column_range(self._h, int(d), _ptr(x), int(n), _ptr(lo), _ptr(hi),
                                     int(flags | x_flags(x))))

    def histogram(self, x, edges, first_denom, counts, flags=0):
        """np.histogram counts per column: x (n, d), edges (d, bins+1), first_denom
        (d, 2), counts (d, bins) int64 -- all host or all device (LGS_DEVICE_PTRS)."""
        n, d = x.shape
        bins = edges.shape[1] - 1
        if tuple(edges.shape) != (d, bins + 1) or tuple(first_denom.shape) != (d, 2) or \
                tuple(counts.shape) != (d, bins):
            raise ValueError("histogram: edges (d, bins+1), first_denom (d, 2), counts (d, bins)")
        _check_bufs(flags, self.device, ((edges, "float64", "edges"), (first_denom, "float64", "first_denom"),
                                         (counts, "int64", "counts")))
        self._ck(self._L.lgs_histogram(self._h, int(d), _ptr(x), int(n), int(bins), _ptr(edges),
                                  _ptr(first_denom), _ptr(counts), int(flags | x_flags(x))))

    # ---------------------------------------------------------------- timing / info
    def timing_enable(self, on=True):
        self._ck(self._L.lgs_timing_enable(self._h, 1 if on else 0))

    def timing_get(self, kernel):
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        self._ck(self._L.lgs_timing_get(self._h, int(kernel), ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def resolved(self, reset=False):
        """Decisions the certificate did not cover and that were redone at the
        reference-order mean (LGS_COUNTER_RESOLVED), since creation / the last reset."""
        v = ctypes.c_uint64(0)
        self._ck(self._L.lgs_counter(self._h, LGS_COUNTER_RESOLVED, 1 if reset else 0, ctypes.byref(v)))
        return v.value

    def fallbacks(self, reset=False):
        """Klein launches redone with a wider store / the fp64 far field (LGS_COUNTER_FALLBACK)."""
        v = ctypes.c_uint64(0)
        self._ck(self._L.lgs_counter(self._h, LGS_COUNTER_FALLBACK, 1 if reset else 0, ctypes.byref(v)))
        return v.value

    def counter(self, which, reset=False):
        """lgs_counter: one of the LGS_COUNTER_* event counts since creation / the last reset."""
        v = ctypes.c_uint64(0)
        self._ck(self._L.lgs_counter(self._h, int(which), 1 if reset else 0, ctypes.byref(v)))
        return v.value

    def device_info(self):
        buf = ctypes.create_string_buffer(256)
        ncu = ctypes.c_int(0)
        mem = ctypes.c_int64(0)
        self._ck(self._L.lgs_device_info(self._h, buf, 256, ctypes.byref(ncu), ctypes.byref(mem)))
        return {"name": buf.value.decode(), "n_cu": ncu.value, "hbm_bytes": mem.value}


def version() -> int:
    return load_library().lgs_version()
