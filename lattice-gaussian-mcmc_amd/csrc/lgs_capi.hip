// lgs_capi.hip -- the C-ABI of include/lgs.h: context, device-resident basis,
// batching, host<->device staging and error reporting around the kernels of
// lgs_kernels.hip.  No CPU compute path exists: every sample is drawn on the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <climits>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lgs.h"
#include "lgs_kernels.h"
#include "lgs_szc_host.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return fail(LGS_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                             \
    } while (0)

// Test / experiment switches read from the environment exist only in builds with
// -DLGS_TEST_HOOKS (liblgs_hip_hooks.so, the A/B variants of tools/build_variant.sh):
// in the product library hook() is a constant nullptr and every such branch folds
// away, so nothing in a user's environment changes what the library computes.  The
// real options are lgs_create_ex's arguments.
#ifdef LGS_TEST_HOOKS
static const char* hook(const char* name) { return getenv(name); }
#else
static constexpr const char* hook(const char*) { return nullptr; }
#endif
static bool hook_is(const char* name, int v) {
    const char* e = hook(name);
    return e && atoi(e) == v;
}

// (hooks build) LGS_TEST_NOMEM_ABOVE=bytes: every device allocation above that size fails,
// as on a full device (tests/test_gpu_edges.py: lgs_imhk's halving of its block)
#ifdef LGS_TEST_HOOKS
static size_t test_nomem_above() {  // (read per allocation: tests set and clear it)
    const char* e = hook("LGS_TEST_NOMEM_ABOVE");
    return e ? (size_t)atoll(e) : 0;
}
#endif

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    int reserve(size_t need) {
        if (need <= bytes) return LGS_OK;
        if (p) {
            (void)hipFree(p);
            p = nullptr;
            bytes = 0;
        }
        if (need == 0) return LGS_OK;
#ifdef LGS_TEST_HOOKS
        if (test_nomem_above() && need > test_nomem_above())
            return fail(LGS_ERR_NOMEM, "hipMalloc(%zu) refused (LGS_TEST_NOMEM_ABOVE)", need);
#endif
        hipError_t e = hipMalloc(&p, need);
        if (e != hipSuccess) {
            p = nullptr;
            return fail(LGS_ERR_NOMEM, "hipMalloc(%zu) failed: %s", need, hipGetErrorString(e));
        }
        bytes = need;
        return LGS_OK;
    }
    void release() {  // (hipFree waits for the device's work on it)
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* as() const {
        return (T*)p;
    }
};

struct Timer {
    int kernel;
    hipEvent_t a, b;
    bool spec = false;  // a look-ahead launch's: dropped if the launch is discarded
};

struct BzCall {  // an int8-digit B z launch, replayed in fp64 if a digit overflowed
    const void* Z;
    int zb;
    int64_t ldz, n;
    double* V;
    int64_t rb, rstride, roff;
    const int64_t* sel;  // nullable: sample s reads column sel[s] of Z
    double* VN;          // nullable: ||v||^2 of rows q < vn_n (same row index, ld 1)
    int64_t vn_n;
};

}  // namespace

struct lgs_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    // basis
    int64_t d = 0;
    double sigma = 0;
    int precision = 10;
    uint32_t basis_flags = 0;
    int panel = 32;
    bool has_B = false;
    DevBuf R, RP, RC, BT, coord;  // coord: cp | rii | sig | sig_ref | lterm | irii | ros | isr
    DevBuf CREC, RX;              // 32-row panels: per-coordinate records, coupling blocks
    DevBuf CERT;                  // per coordinate {Ca, Cb}: decision certificate
    uint64_t n_resolved = 0;      // sub-panel verifications of uncertified decisions
    // certified Wang-Ling accept decisions (imhk_accept_cert_kernel): R transposed,
    // the per-proposal weight bounds, the running maximum bound (device word, reset
    // by lgs_set_basis), counters of resolved decisions and of recomputed draws that
    // did not reproduce the stored z (0 unless a bug)
    DevBuf RT, LWE, EMAX;
    DevBuf QZ2;            // per 32-row panel: the q-panel skip's bound on ||z_W||^2 (klein_mfma_kernel)
    bool has_qz2 = false;
    uint64_t n_accept_resolved = 0, n_wl_mismatch = 0;
    uint64_t n_qskip = 0;  // (wave, panel) pairs decided by the q-panel skip
    uint64_t n_fallback = 0;      // Klein launches redone with a wider store / fp64 far field
    // 32-row-panel kernels: the certificate's bound on sum_j |z_j| of a sample (an
    // estimate from the basis, then twice the largest sum seen; a sample exceeding it
    // is replayed in the reference's order, so the cap only affects speed)
    double z1cap = 0.0, z1seen = 0.0;
    unsigned int resolved_seen = 0;  // run_klein_store: the resolved word after the call's last launch
    DevBuf RD, RDOFF;             // int8-digit far field: R digit fragments, panel offsets
    bool has_rd = false, oz_off = false;  // oz_off: a |z| > 32767 was seen (sticky)
    DevBuf H16, F0;               // int8-digit far field scratch: coefficient history, tile-0 sums
    DevBuf ZNZ;                   // per history block and lane: any nonzero z (B z's chunk skipping)
    DevBuf CLIVE;                 // per wave and 64-coordinate chunk: any nonzero z (bits; B z)
    DevBuf VNP;                   // B z's per-tile partial sums of ||v||^2 (lgs_imhk_ex vnorm2_samples)
    DevBuf LAGP;                  // lag-sum partials per (lag, chain) (lgs_imhk_ex lag_L)
    // the last Klein launch's history, valid for columns [0, cols) of the store Z it
    // wrote (B z reads its digits from there); reset by every Klein launch
    struct {
        const void* Z = nullptr;
        int64_t lanes = 0, cols = 0;
        const unsigned int* clive = nullptr;  // its per-wave chunk bits (nullable)
        int64_t clive_ld = 0;
    } hist;
    DevBuf Bd;                    // int8 digit planes of B (hi | lo), [row][k], k padded to 64
    DevBuf kchunk, koff;          // per 128-row tile of B: the 64-column chunks with a non-zero digit
    bool bz_mom_ok = false;       // every 64-column chunk has an owner tile (B z can sum the moments)
    DevBuf MP;                    // B z's moment partials per (64-row tile, coordinate)
    DevBuf etab;                  // SampleZ erf/exp table (lgs_device.h erf_gauss)
    DevBuf etab2;                 // its Taylor-coefficient form (lgs_device.h CoefTab)
    DevBuf szc;                   // per-coordinate SampleZ constants (lgs_kernels.h kSzc*)
    bool libm_samplez = false;    // LGS_SAMPLEZ_LIBM=1: ocml erf/exp/erfinv path instead
    bool has_Bi8 = false;
    int64_t bd_rows = 0, bd_cols = 0;
    std::vector<BzCall> pending_i8;
    // an int8 B z whose fp64 replay was enqueued on the device, gated on the digit-range
    // flag (run_bz device_replay): settle_bz then only clears that flag bit
    bool i8_dev_replay = false;
    // scratch
    DevBuf Z, LW, V, sel, fsel, cnt, ccnt, flags, stage_a, stage_b, stage_c, stage_d, stage_e,
        stage_f, stage_g, stage_h, stage_i, vs;
    int64_t max_props = 1 << 18;
    bool max_props_user = false;  // lgs_create_ex's cap (else set per basis, lgs_set_basis)
    bool no_pipe = false, no_look = false, no_qskip = false, no_cu_split = false;  // lgs_create_ex ctx_flags
    int zint = 2;  // internal coefficient store width (bytes): 16-bit, sticky 32-bit on overflow; LGS_ZINT=4 forces 32-bit
    // timing
    bool timing = false;
    double t_ms[7] = {0, 0, 0, 0, 0, 0, 0};
    int64_t t_n[7] = {0, 0, 0, 0, 0, 0, 0};
    // diagnostics scratch (lgs_series_stats / lgs_gram / lgs_jump_distance / lgs_marginal_tvd)
    DevBuf dg_x, dg_y, dg_out, dg_a, dg_b, dg_c, dg_t;
    // decoding frame (lgs_set_decoder): Q of the QR and (B^{-1})^T, row-major d x d
    DevBuf DQ, DBIT;
    bool has_q = false, has_binv = false;
    std::vector<Timer> pending;
    std::vector<hipEvent_t> pool;
    // lgs_imhk on a caller's stream (early check): the flag words as of a block's
    // abort producers, copied into pinned host memory, and the event after that copy
    unsigned int* fw_host = nullptr;
    hipEvent_t fw_ev = nullptr;
    // Pipelined blocks (lgs_imhk with the early check): each block's Klein launch runs
    // on kstream into one of two buffer sets (proposal store, weights, int16 history,
    // zero flags, flag words), so the next block's -- or the next call's -- launch
    // runs beside this block's accept / moments / B z on the caller's stream (IMHK
    // proposals do not depend on the chain state).  ev_free: recorded on the caller's
    // stream after the set's last reader; the set's next Klein launch waits for it.
    struct BlockSet {
        DevBuf Z, LW, H16, ZNZ, CLIVE, flags;
        hipEvent_t ev_free = nullptr;
        bool free_recorded = false;
    } bset[3];
    int bset_next = 0;
    int nsets = 2;  // buffer sets in rotation (LGS_PIPE_SETS=3: three, fixed at the first pipelined call)
    bool kstream_sets_fixed = false;
    hipStream_t kstream = nullptr;
    // CU split (lgs_imhk, pipelined): kstream is kstream_full (every CU) or kstream_split
    // (its queue masked off 1/8 of the CUs).  cu_split: 0 undecided (the first pipelined
    // Klein launch is timed on kstream_full, kt0 / kt1), 1 split, 2 every CU.
    hipStream_t kstream_full = nullptr, kstream_split = nullptr;
    int cu_split = 0;
    int kstream_cus = 0;  // CUs in kstream's mask (0: all)
    int split_cus = 0;    // CUs in kstream_split's mask
    hipEvent_t kt0 = nullptr, kt1 = nullptr;
    bool kt_pending = false;
    double kt_bz_ms = 0.0;  // the timed block's B z store estimate
    hipEvent_t ev_klein = nullptr;
    // Look-ahead: at the end of a pipelined call, the Klein launch of the next call's
    // first block as this call predicts it (same seed, chains, steps per call, store;
    // the counters continue) is enqueued on kstream into the next set, so the Klein
    // stream never waits for the host's turnaround between calls.  The next call uses
    // it when its first block matches the prediction, else discards it (it writes
    // only that set).  Proposals are counter-addressed: a launch made early is the
    // same launch.
    struct Spec {
        bool valid = false;
        uint64_t seed = 0, chain0 = 0, step0 = 0;
        int64_t nc = 0, Tb = 0, ldzb = 0;
        int zb = 0, j = 0;
        bool wl = false, exact = false, oz = false;
        decltype(hist) h;
        hipEvent_t ev = nullptr;  // recorded on kstream behind the launch
    } spec;
};

namespace {

int check_ctx(lgs_ctx* c, bool need_basis = true) {
    if (!c) return fail(LGS_ERR_INVALID, "null context");
    if (need_basis && c->d <= 0) return fail(LGS_ERR_STATE, "no basis loaded (lgs_set_basis)");
    HIP_TRY(hipSetDevice(c->device));
    return LGS_OK;
}

hipEvent_t get_event(lgs_ctx* c) {
    if (!c->pool.empty()) {
        hipEvent_t e = c->pool.back();
        c->pool.pop_back();
        return e;
    }
    // no system-scope fence: a timing event must not add an L2 writeback to the
    // stream (measured +0.6 ms on the Klein launch with the default flags)
    hipEvent_t e = nullptr;
    (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    return e;
}

struct Scope {  // times one launch when timing is enabled
    lgs_ctx* c;
    int k;
    hipEvent_t a = nullptr;
    Scope(lgs_ctx* c_, int k_) : c(c_), k(k_) {
        if (c->timing) {
            a = get_event(c);
            (void)hipEventRecord(a, c->stream);
        }
    }
    ~Scope() {
        if (c->timing && a) {
            hipEvent_t b = get_event(c);
            (void)hipEventRecord(b, c->stream);
            c->pending.push_back({k, a, b});
        }
    }
};

int run_bz_fp64(lgs_ctx* c, const BzCall& b);

void swap_buf(DevBuf& a, DevBuf& b) {
    std::swap(a.p, b.p);
    std::swap(a.bytes, b.bytes);
}

// A pipelined block's buffer set swapped into the context's working buffers (which
// every launch path uses), and back on every exit from the block.  The flag words
// first: the block's initial draws (into the context's own store) already report
// into them; then the store, for the block's own Klein launch and its dependants.
struct SetSwap {
    lgs_ctx* c = nullptr;
    int j = -1;
    bool flags_in = false, store_in = false;
    void swap_flags() {
        swap_buf(c->flags, c->bset[j].flags);
        flags_in = !flags_in;
    }
    void swap_store() {
        auto& s = c->bset[j];
        swap_buf(c->Z, s.Z);
        swap_buf(c->LW, s.LW);
        swap_buf(c->H16, s.H16);
        swap_buf(c->ZNZ, s.ZNZ);
        swap_buf(c->CLIVE, s.CLIVE);
        store_in = !store_in;
    }
    void restore() {
        if (j < 0) return;
        if (store_in) swap_store();
        if (flags_in) swap_flags();
    }
    // The block is over, on its normal path or an error return (a finish() error such
    // as LGS_ERR_OVERFLOW / LGS_ERR_NONFINITE leaves the block's accept, B z, moments and
    // gathers enqueued on the caller's stream, still reading the set): the buffers go
    // back, and the set's free event is recorded behind whatever the block enqueued, so
    // the set's next Klein launch (kstream) waits for those readers in every case.
    bool record = true;  // (the look-ahead launch: no reader of its own on the caller's stream)
    void release() {
        if (j < 0) return;
        restore();
        if (record) {
            (void)hipEventRecord(c->bset[j].ev_free, c->stream);
            c->bset[j].free_recorded = true;
        }
        j = -1;
    }
    ~SetSwap() { release(); }
};

// The CU split's decision (lgs_ctx::cu_split), once, after the first pipelined call
// whose timed Klein launch (every CU, kt0 -> kt1) has finished: the split costs the
// Klein launches cu_res / split_cus of their time (1/7) and hides the previous block's
// B z behind them, so it is taken when that block's B z -- its lattice-point stores,
// 8 d bytes per kept proposal at the ~4.6 TB/s bz_i8_kernel reaches on MI355X -- is the
// larger.  Measured (bench, same box, profiles/r06bc_bench_cusplit_ab.log): C3 0.26 of
// the Klein time, split +3.0 %; C4 0.16, +1.6 %; C5 0.13, -3.4 %; C2 0.09, -3.6 %.
constexpr double kBzStoreBytesPerMs = 4.6e9;
static int split_decide(lgs_ctx* c) {
    if (c->cu_split != 0 || !c->kt_pending || hipEventQuery(c->kt1) != hipSuccess) return LGS_OK;
    c->kt_pending = false;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, c->kt0, c->kt1) != hipSuccess || !(ms > 0.f)) return LGS_OK;  // (timed again)
    const int ncu = c->split_cus * 8 / 7;
    const double cost = (double)ms * (double)(ncu - c->split_cus) / (double)c->split_cus;
    if (c->kt_bz_ms > cost) {
        HIP_TRY(hipStreamSynchronize(c->kstream_full));  // (idle but for an early look-ahead launch)
        c->kstream = c->kstream_split;
        c->kstream_cus = c->split_cus;
        c->cu_split = 1;
    } else {
        c->cu_split = 2;
    }
    return LGS_OK;
}

// Drops a look-ahead Klein launch (lgs_ctx::Spec): waits for it and clears the flag
// words it wrote into its set.
int spec_discard(lgs_ctx* c) {
    if (!c->spec.valid) return LGS_OK;
    c->spec.valid = false;
    HIP_TRY(hipStreamSynchronize(c->kstream));
    HIP_TRY(hipMemset(c->bset[c->spec.j].flags.p, 0, 4 * lgs::kFlagWords));
    // its launch timers do not count (the launch's work is thrown away)
    size_t keep = 0;
    for (auto& t : c->pending) {
        if (t.spec) {
            c->pool.push_back(t.a);
            c->pool.push_back(t.b);
        } else {
            c->pending[keep++] = t;
        }
    }
    c->pending.resize(keep);
    return LGS_OK;
}

// Wait for the stream; if an int8-digit B z saw a coefficient beyond two digits,
// replay the pending B z launches with the fp64 kernel.  Must run before any
// copy that consumes their output.
// f0_known: the caller has synchronised and read flag word 0 already (*f0_known).
int settle_bz(lgs_ctx* c, const unsigned int* f0_known = nullptr) {
    if (!f0_known) HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->pending_i8.empty() && !c->i8_dev_replay) return LGS_OK;
    {
        unsigned int f0 = 0;
        if (f0_known)
            f0 = *f0_known;
        else
            HIP_TRY(hipMemcpy(&f0, c->flags.p, sizeof(f0), hipMemcpyDeviceToHost));
        if (f0 & lgs::kFlagI8Range) {  // coefficients beyond two int8 digits: redo in fp64
            for (const auto& b : c->pending_i8) {
                int rc = run_bz_fp64(c, b);
                if (rc) return rc;
            }
            const unsigned int keep = f0 & ~lgs::kFlagI8Range;
            HIP_TRY(hipMemcpyAsync(c->flags.p, &keep, sizeof(keep), hipMemcpyHostToDevice, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
        }
        c->pending_i8.clear();
        c->i8_dev_replay = false;
    }
    return LGS_OK;
}

// flags buffer (device, 32 bytes): [0] kernel flag bits, [1] kFlagWordResolved
// counter, [2..3] the largest sum |z_j| of a Klein launch (fp64 bits, atomicMax),
// [4] lgs_imhk: some chain needs its initial draw, [5] lgs_imhk: the resolved
// counter before the block's own Klein launch (a checkpoint taken by init_apply)
using lgs::kFlagWordUninit;
using lgs::kFlagWordCheckpoint;

// Folds the counters of a finished stretch of launches into the context: the
// resolved count, and the certificate's cap on sum |z_j| = twice the larger of the
// largest sums of the last two stretches (the basis-derived bound of lgs_set_basis
// only until a launch has been seen): a tight cap keeps the bound dmu small, and
// one launch with outlying |z| no longer inflates it for good (a sum above the cap
// only forces that sub-panel's verification).
void fold_counters(lgs_ctx* c, const unsigned int* fw) {
    c->n_resolved += fw[1];
    double z1;
    memcpy(&z1, fw + 2, sizeof(z1));
    if (z1 > 0.0) {
        c->z1cap = 2.0 * std::max(z1, c->z1seen);
        c->z1seen = z1;
    }
}

// Folds the finished launch timers into the context's totals; a timer whose end
// event is still pending (the early check leaves a block's later launches running)
// stays for a later call or lgs_timing_get.
void fold_timers(lgs_ctx* c) {
    size_t keep = 0;
    for (auto& t : c->pending) {
        if (t.spec || hipEventQuery(t.b) != hipSuccess) {  // (a look-ahead's: until used or discarded)
            c->pending[keep++] = t;
            continue;
        }
        float ms = 0;
        if (hipEventElapsedTime(&ms, t.a, t.b) == hipSuccess) {
            c->t_ms[t.kernel] += ms;
            c->t_n[t.kernel] += 1;
        }
        c->pool.push_back(t.a);
        c->pool.push_back(t.b);
    }
    c->pending.resize(keep);
}

// fw_known: the caller has synchronised and read the flag words (one device-to-host
// copy per call instead of one per check: each is a round trip the GPU idles through).
// clear_all: reset every flag word, word 0 included, behind the work already enqueued
// (the early check: word 0 may still receive the digit-range bit of a B z whose
// device-gated replay follows it).
int finish(lgs_ctx* c, const unsigned int* fw_known = nullptr, bool clear_all = false) {  // sync, fold timers, report kernel flags
    int rc0 = settle_bz(c, fw_known);
    if (rc0) return rc0;
    fold_timers(c);
    unsigned int fw[lgs::kFlagWords] = {};
    if (fw_known)
        memcpy(fw, fw_known, sizeof(fw));
    else
        HIP_TRY(hipMemcpy(fw, c->flags.p, sizeof(fw), hipMemcpyDeviceToHost));
    const unsigned int f = fw[0];
    c->resolved_seen = 0;
    if (fw[1] || fw[2] || fw[3])
        fold_counters(c, fw);
    c->n_accept_resolved += fw[lgs::kFlagWordAcceptResolved];
    c->n_wl_mismatch += fw[lgs::kFlagWordWLMismatch];
    c->n_qskip += fw[lgs::kFlagWordQSkip];
    bool any = false;
    for (int k = 1; k < lgs::kFlagWords; ++k) any |= fw[k] != 0;
    if (clear_all)
        HIP_TRY(hipMemsetAsync(c->flags.p, 0, lgs::kFlagWords * sizeof(unsigned int), c->stream));
    else if (any)  // ordered before the next launches
        HIP_TRY(hipMemsetAsync((unsigned int*)c->flags.p + 1, 0, (lgs::kFlagWords - 1) * sizeof(unsigned int),
                               c->stream));
    if (f & lgs::kFlagNonFinite)
        return fail(LGS_ERR_NONFINITE, "non-finite conditional mean (reference raises ValueError)");
    if (f & lgs::kFlagOverflow)
        return fail(LGS_ERR_OVERFLOW, "coefficient |z| >= 2^31: rerun with LGS_Z64");
    return LGS_OK;
}

// One synchronisation for a stretch of lgs_imhk launches enqueued without waiting
// (a Klein launch and its dependants).  If the Klein launch overflowed its 16-bit
// store / int16 history, or a carried-in state did not fit the 16-bit store
// (kAbortMask), the dependants returned without touching the caller's state: the
// attempt is discarded (its B z launches, its verification count beyond the
// checkpoint, its |z| maximum), the context switches to the wider store / the fp64
// far field, and redo is set.  Otherwise the usual finish().
//
// early (lgs_imhk on a caller's stream): the flag words were copied into fw_host
// right after the block's abort producers (its Klein launches, the carried-in
// states) and the block's later launches are already enqueued; wait for that copy
// only, so the caller's next work is enqueued while they run.  Those later launches
// write no flag the host reads (reference weights: no accept counters; B z's digit
// range is replayed on the device), and every flag word is reset behind them.
int finish_or_redo(lgs_ctx* c, bool oz_used, int& zb, bool& redo, bool early = false) {
    redo = false;
    unsigned int fw[lgs::kFlagWords];
    if (early) {
        HIP_TRY(hipEventSynchronize(c->fw_ev));
        memcpy(fw, c->fw_host, sizeof(fw));
    } else {
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(hipMemcpy(fw, c->flags.p, sizeof(fw), hipMemcpyDeviceToHost));
    }
    if (!(fw[0] & lgs::kAbortMask)) return finish(c, fw, early);
    c->pending_i8.clear();
    c->i8_dev_replay = false;
    for (auto& t : c->pending) {  // the aborted attempt's timers are not kept
        c->pool.push_back(t.a);
        c->pool.push_back(t.b);
    }
    c->pending.clear();
    c->n_fallback += 1;
    c->n_resolved += fw[kFlagWordCheckpoint];
    if (fw[0] & lgs::kFlagOverflow16) {
        if (zb == 2) c->zint = 4;
        if (oz_used) c->oz_off = true;
    }
    if (fw[0] & lgs::kFlagCarry16) c->zint = 4;
    if (zb == 2) zb = c->zint;
    HIP_TRY(hipMemsetAsync(c->flags.p, 0, 4 * lgs::kFlagWords, c->stream));
    redo = true;
    return LGS_OK;
}

int reset_flags(lgs_ctx* c) {
    int rc = c->flags.reserve(4 * lgs::kFlagWords);
    if (rc) return rc;
    c->resolved_seen = 0;
    HIP_TRY(hipMemsetAsync(c->flags.p, 0, 4 * lgs::kFlagWords, c->stream));
    return LGS_OK;
}

lgs::KleinArgs base_args(lgs_ctx* c, uint64_t seed) {
    lgs::KleinArgs a{};
    const double* co = c->coord.as<double>();
    const int64_t d = c->d;
    a.d = (int)d;
    a.precision = c->precision;
    a.linear_probs = (c->basis_flags & LGS_BASIS_LINEAR_PROBS) ? 1 : 0;
    a.cp = co;
    a.rii = co + d;
    a.sig = co + 2 * d;
    a.sig_ref = co + 3 * d;
    a.lterm = co + 4 * d;
    a.irii = co + 5 * d;
    a.ros = co + 6 * d;
    a.isr = co + 7 * d;
    a.sigma = c->sigma;
    a.seed = seed;
    a.flags = c->flags.as<unsigned int>();
    a.etab = c->libm_samplez ? nullptr : c->etab.as<double>();
    a.etab2 = c->etab2.as<double>();
    a.szc = c->libm_samplez ? nullptr : c->szc.as<double>();
    a.crec = c->CREC.as<double>();
    a.rx = c->RX.as<double>();
    a.R = c->R.as<double>();
    a.cert = c->CERT.as<double>();
    a.z1cap = c->z1cap;
    // test hook: scale the certificate's cap on sum |z_j| (a cap below the actual sums
    // forces every 32-row-panel sub-panel through the verification / replay path)
    if (const char* s = hook("LGS_TEST_Z1CAP_SCALE")) a.z1cap *= atof(s);
    a.z1max = (unsigned long long*)c->flags.as<unsigned int>() + 1;
    const bool no_qskip = c->no_qskip || hook_is("LGS_NO_QSKIP", 1);  // (LGS_CTX_NO_QSKIP: A/B)
    a.qz2 = c->has_qz2 && !no_qskip ? c->QZ2.as<double>() : nullptr;
    return a;
}

// The int8-digit far field's per-launch buffers for n proposals (the sizes run_klein
// reserves; pre-reserved by lgs_imhk so that an allocation failure halves its block).
int reserve_oz(lgs_ctx* c, DevBuf& H16, DevBuf& ZNZ, DevBuf& CLIVE, int64_t n) {
    if (!(c->panel == 32 && c->has_rd)) return LGS_OK;
    const int shift = (int)((16 - c->d % 16) % 16);
    const int64_t lanes = (n + 63) / 64 * 64;
    const int64_t blocks = (c->d + shift) / 16 + 5;
    int rc = H16.reserve((size_t)blocks * lanes * 32);
    if (!rc) rc = ZNZ.reserve((size_t)blocks * lanes);
    if (!rc && c->d % 16 == 0) rc = CLIVE.reserve((size_t)((c->d + 2047) / 2048 * (lanes / 64)) * 4);
    return rc;
}

// Kernel choice: exact order on request; otherwise the MFMA kernel when the launch
// is whole waves with aligned coefficient rows (32-row panels: int8-digit far field
// unless disabled), else the VALU panel kernel.  LGS_KERNEL=valu|mfma|mfma64|exact
// overrides (mfma64: fp64 MFMA far field).  Returns whether the int8-digit far
// field was used.
int run_klein(lgs_ctx* c, lgs::KleinArgs& a, bool exact, bool wl, int zb, void* Z, bool& used_oz) {
    Scope s(c, a.gate ? 6 : 0);  // gated launches (lgs_imhk's initial draws) on their own timer
    static const char* force = hook("LGS_KERNEL");
    int kernel = lgs::kKernelValu;
    used_oz = false;
    c->hist.Z = nullptr;
    if (exact || (force && strcmp(force, "exact") == 0))
        kernel = lgs::kKernelExact;
    else if (!(force && strcmp(force, "valu") == 0) && a.n % 64 == 0 && a.ldz % 4 == 0 &&
             ((uintptr_t)Z % 16) == 0)
        kernel = lgs::kKernelMfma;
    a.rd = nullptr;
    // (the int8-digit far field synchronises the block per step: whole blocks only)
    if (kernel == lgs::kKernelMfma && c->panel == 32 && c->has_rd && !c->oz_off && a.n % 256 == 0 &&
        !(force && strcmp(force, "mfma64") == 0)) {
        const int shift = (int)((16 - c->d % 16) % 16);
        const int64_t lanes = (a.n + 63) / 64 * 64;
        const int64_t blocks = (c->d + shift) / 16 + 5;  // + one 64-column chunk of padding
        int rc = c->H16.reserve((size_t)blocks * lanes * 32);
        if (rc) return rc;
        if ((rc = c->ZNZ.reserve((size_t)blocks * lanes))) return rc;
        a.znz = c->ZNZ.as<uint8_t>();
#ifndef LGS_NEAR_UNROLLED
        if (c->d % 16 == 0) {  // per-wave chunk bits for B z (zeroed: the kernel ORs into them)
            const int64_t words = (c->d + 2047) / 2048 * (lanes / 64);
            if ((rc = c->CLIVE.reserve((size_t)words * 4))) return rc;
            HIP_TRY(hipMemsetAsync(c->CLIVE.p, 0, (size_t)words * 4, c->stream));
            a.clive = c->CLIVE.as<unsigned int>();
            a.clive_ld = lanes / 64;
        }
#endif
        a.rd = c->RD.as<int8_t>();
        a.rd_off = c->RDOFF.as<int64_t>();
        a.h16 = c->H16.as<int16_t>();
        a.h16_shift = shift;
        a.h16_lanes = lanes;
        used_oz = true;
    }
    HIP_TRY(lgs::launch::klein(a, c->R.as<double>(), c->RP.as<double>(), c->RC.as<double>(),
                               c->panel, kernel, wl, zb, Z, c->stream));
    return LGS_OK;
}

// Klein launch into an internal coefficient store of width zb.  A coefficient
// beyond int16 (a 16-bit store, or the int16 history of the int8-digit far field)
// redoes the launch -- same counters, same samples -- at 32 bits / with the fp64
// far field, and the context keeps that choice.  deferred (lgs_imhk): no wait
// here; the caller's single synchronisation (finish_or_redo) makes that check.
int run_klein_store(lgs_ctx* c, lgs::KleinArgs& a, bool exact, bool wl, int& zb, void* Z, bool deferred,
                    bool* oz_out = nullptr) {
    bool oz = false;
    int rc = run_klein(c, a, exact, wl, zb, Z, oz);
    if (oz_out) *oz_out = oz;
    if (oz) {
        c->hist.Z = Z;
        c->hist.lanes = (a.n + 63) / 64 * 64;
        c->hist.cols = a.n;
        c->hist.clive = a.clive;
        c->hist.clive_ld = a.clive_ld;
    }
    if (rc || deferred || (zb != 2 && !oz)) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    unsigned int f[2] = {0, 0};
    HIP_TRY(hipMemcpy(f, c->flags.p, sizeof(f), hipMemcpyDeviceToHost));
    if (!(f[0] & lgs::kFlagOverflow16)) {
        c->resolved_seen = f[1];  // the count up to and including this launch
        return LGS_OK;
    }
    // discard this launch's verification count: keep what earlier launches of the
    // call had counted (folded into the context now, the word restarts at 0)
    c->n_resolved += c->resolved_seen;
    c->resolved_seen = 0;
    f[0] &= ~lgs::kFlagOverflow16;
    f[1] = 0;
    c->n_fallback += 1;
    HIP_TRY(hipMemcpy(c->flags.p, f, sizeof(f), hipMemcpyHostToDevice));
    if (zb == 2) {
        c->zint = 4;
        zb = 4;
    }
    if (oz) c->oz_off = true;
    c->hist.Z = nullptr;
    rc = run_klein(c, a, exact, wl, zb, Z, oz);
    if (oz_out) *oz_out = oz;
    return rc;
}

int run_bz_fp64(lgs_ctx* c, const BzCall& b) {
    Scope s(c, 1);
    HIP_TRY(lgs::launch::bz(b.Z, b.zb, b.ldz, b.sel, c->BT.as<double>(), (int)c->d, b.n, b.V, c->d, b.rb,
                            b.rstride, b.roff, c->stream));
    if (b.VN) HIP_TRY(lgs::launch::vnorm2_rows(b.V, (int)c->d, b.vn_n, b.rb, b.rstride, b.roff, b.VN, c->stream));
    return LGS_OK;
}

// v = B z: exact int8-digit MFMA kernel for integer bases (fp64 replay on digit
// overflow, see finish()), fp64 MFMA kernel otherwise.  LGS_BZ_FP64=1 forces fp64.
// after_klein: Z holds the output of the last Klein launch (its int16 history is
// then a valid source of the digits for the columns that launch wrote).
int run_bz(lgs_ctx* c, const void* Z, int zb, int64_t ldz, int64_t n, double* V,
           int64_t rb = 0, int64_t rstride = 0, int64_t roff = 0, const int64_t* sel = nullptr,
           bool after_klein = false, const unsigned int* abort = nullptr, double* VN = nullptr,
           int64_t vn_n = -1, bool device_replay = false, unsigned long long* MP = nullptr,
           int64_t mp_ld = 0, unsigned int* MPL = nullptr) {
    if (!c->has_B) return fail(LGS_ERR_STATE, "lattice points need B (lgs_set_basis B != NULL)");
    if (vn_n < 0 || vn_n > n) vn_n = n;  // ||v||^2 of the leading vn_n rows only
    if (vn_n == 0) VN = nullptr;
    BzCall b{Z, zb, ldz, n, V, rb > 0 ? rb : n, rstride, roff, sel, VN, vn_n};
    static const bool force64 = hook_is("LGS_BZ_FP64", 1);
    if (!c->has_Bi8 || force64) {
        Scope s(c, 1);
        HIP_TRY(lgs::launch::bz(b.Z, b.zb, b.ldz, b.sel, c->BT.as<double>(), (int)c->d, b.n, b.V, c->d, b.rb,
                                b.rstride, b.roff, c->stream, abort));
        if (VN) HIP_TRY(lgs::launch::vnorm2_rows(b.V, (int)c->d, vn_n, b.rb, b.rstride, b.roff, VN, c->stream));
        return LGS_OK;
    }
    Scope s(c, 1);
    const int8_t* hi = c->Bd.as<int8_t>();
    const int8_t* lo = hi + (size_t)c->bd_rows * c->bd_cols;
    // timing probes only (wrong outputs): LGS_DIAG_BZ=1 drops the ||v||^2 rows, 2 the
    // selections (row q reads proposal q), 3 both
    static const int diag_bz = hook("LGS_DIAG_BZ") ? atoi(hook("LGS_DIAG_BZ")) : 0;
    if (diag_bz & 1) VN = nullptr;
    if (diag_bz & 2) sel = nullptr;
    double* VNP = nullptr;
    if (VN) {
        const int rc = c->VNP.reserve((size_t)2 * ((c->d + lgs::kBzBN - 1) / lgs::kBzBN) * vn_n * 8);
        if (rc) return rc;
        VNP = c->VNP.as<double>();
    }
    HIP_TRY(lgs::launch::bz_i8(Z, zb, ldz, sel, c->kchunk.as<int>(), c->koff.as<int>(), hi, lo,
                               (int)c->bd_cols, (int)c->d, n, V, c->d, b.rb,
                               b.rstride, b.roff, c->flags.as<unsigned int>(),
                               after_klein && c->hist.Z == Z && Z ? c->H16.as<int16_t>() : nullptr, c->hist.lanes,
                               c->hist.cols, c->stream, abort, c->ZNZ.as<uint8_t>(),
                               after_klein && c->hist.Z == Z && Z ? c->hist.clive : nullptr, c->hist.clive_ld,
                               VNP, vn_n, MP, mp_ld, MPL));
    if (VN) HIP_TRY(lgs::launch::vnorm2_reduce(VNP, (int)c->d, vn_n, b.rb, b.rstride, b.roff, VN, c->stream, abort));
    if (device_replay) {  // the fp64 replay enqueued now, run only if the digit-range flag is set
        c->i8_dev_replay = true;
        const unsigned int* need = c->flags.as<unsigned int>();
        HIP_TRY(lgs::launch::bz(b.Z, b.zb, b.ldz, b.sel, c->BT.as<double>(), (int)c->d, b.n, b.V, c->d, b.rb,
                                b.rstride, b.roff, c->stream, abort, need));
        if (VN)
            HIP_TRY(lgs::launch::vnorm2_rows(b.V, (int)c->d, vn_n, b.rb, b.rstride, b.roff, VN, c->stream, abort,
                                             need));
        return LGS_OK;
    }
    c->pending_i8.push_back(b);
    return LGS_OK;
}

// The look-ahead launch (lgs_ctx::Spec): the next call's first block as this call
// predicts it (same arguments, step counter continued), on kstream into set j --
// right behind the call's last Klein launch, before the call waits for anything, so
// the Klein stream runs back to back.  The context's working buffers, history and
// stream are restored on return.
int lookahead(lgs_ctx* c, int j, uint64_t seed, uint64_t first_chain, uint64_t step0, int64_t nc, int64_t tb,
              bool carry, int zb, bool exact, bool wl) {
    const auto hist = c->hist;
    SetSwap sw;
    sw.c = c;
    sw.j = j;
    sw.record = false;
    sw.swap_flags();
    sw.swap_store();
    const int64_t ldz = nc * tb + (carry ? nc : 0);
    lgs::KleinArgs a = base_args(c, seed);
    a.counter_mode = 1;
    a.chain0 = (uint32_t)first_chain;
    a.step0 = (uint32_t)step0;
    a.nt = tb;
    a.n = nc * tb;
    a.ldz = ldz;
    a.LW = c->LW.as<double>();
    auto& bs = c->bset[j];
    if (bs.free_recorded) HIP_TRY(hipStreamWaitEvent(c->kstream, bs.ev_free, 0));
    const hipStream_t cs = c->stream;
    c->stream = c->kstream;
    int zbs = zb;
    bool oz = false;
    const size_t npend = c->pending.size();
    const int rc = run_klein_store(c, a, exact, wl, zbs, c->Z.p, true, &oz);
    for (size_t k = npend; k < c->pending.size(); ++k) c->pending[k].spec = true;
    c->stream = cs;
    const auto h = c->hist;
    c->hist = hist;
    if (rc) return rc;
    if (!c->spec.ev) HIP_TRY(hipEventCreateWithFlags(&c->spec.ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(c->spec.ev, c->kstream));
    auto& sp = c->spec;
    sp.valid = true;
    sp.seed = seed;
    sp.chain0 = first_chain;
    sp.step0 = step0;
    sp.nc = nc;
    sp.Tb = tb;
    sp.ldzb = ldz;
    sp.zb = zb;
    sp.j = j;
    sp.wl = wl;
    sp.exact = exact;
    sp.oz = oz;
    sp.h = h;
    return LGS_OK;
}

hipMemcpyKind kind_of(bool dev_dst, bool dev_src) {
    if (dev_dst && dev_src) return hipMemcpyDeviceToDevice;
    if (dev_dst) return hipMemcpyHostToDevice;
    if (dev_src) return hipMemcpyDeviceToHost;
    return hipMemcpyHostToHost;
}

}  // namespace

extern "C" {

int lgs_version(void) { return 100; }

const char* lgs_last_error(void) { return g_err.c_str(); }

int lgs_create(lgs_ctx** out, int device) { return lgs_create_ex(out, device, 0, 0); }

int lgs_create_ex(lgs_ctx** out, int device, int64_t max_proposals, uint32_t ctx_flags) {
    if (!out) return fail(LGS_ERR_INVALID, "null out pointer");
    if (max_proposals < 0) return fail(LGS_ERR_INVALID, "max_proposals < 0");
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device < 0 || device >= n)
        return fail(LGS_ERR_INVALID, "device %d out of range (%d devices)", device, n);
    HIP_TRY(hipSetDevice(device));
    lgs_ctx* c = new lgs_ctx();
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return fail(LGS_ERR_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    c->stream = c->own;
    // options (include/lgs.h LGS_CTX_*); the hooks build also takes them from the
    // environment for the A/B tools
    c->panel = (ctx_flags & LGS_CTX_PANEL16) ? 16 : 32;
    c->zint = (ctx_flags & LGS_CTX_STORE32) ? 4 : 2;
    c->libm_samplez = (ctx_flags & LGS_CTX_SAMPLEZ_LIBM) != 0;
    // far field of the 32-row-panel kernel: the exact int8-digit product (default)
    // or fp64 MFMA (LGS_CTX_FAR_FP64)
    c->oz_off = (ctx_flags & LGS_CTX_FAR_FP64) != 0;
    c->no_pipe = (ctx_flags & LGS_CTX_NO_PIPELINE) != 0;
    c->no_look = (ctx_flags & LGS_CTX_NO_LOOKAHEAD) != 0;
    c->no_qskip = (ctx_flags & LGS_CTX_NO_QSKIP) != 0;
    c->no_cu_split = (ctx_flags & LGS_CTX_NO_CU_SPLIT) != 0;
    if (max_proposals > 0) {
        c->max_props = std::max<int64_t>(64, max_proposals);
        c->max_props_user = true;
    }
    if (const char* p = hook("LGS_PANEL")) c->panel = atoi(p) == 16 ? 16 : 32;
    if (const char* z = hook("LGS_ZINT")) c->zint = atoi(z) == 2 ? 2 : 4;
    if (const char* m = hook("LGS_MAX_PROPOSALS")) {
        long long v = atoll(m);
        if (v >= 64) {
            c->max_props = v;
            c->max_props_user = true;
        }
    }
    if (const char* m = hook("LGS_SAMPLEZ_LIBM")) c->libm_samplez = atoi(m) != 0;
    if (const char* m = hook("LGS_FAR")) c->oz_off = strcmp(m, "fp64") == 0;
    {
        // {erf(j/64), exp(-(j/64)^2)}, j = 0..kErfTabLast, rounded from long double.
        std::vector<double> tab(2 * (lgs::kErfTabLast + 1));
        for (int j = 0; j <= lgs::kErfTabLast; ++j) {
            const long double y = (long double)j / 64.0L;
            tab[2 * j] = (double)erfl(y);
            tab[2 * j + 1] = (double)expl(-y * y);
        }
        int rc = c->etab.reserve(tab.size() * 8);
        if (!rc) {
            e = hipMemcpy(c->etab.p, tab.data(), tab.size() * 8, hipMemcpyHostToDevice);
            if (e != hipSuccess) rc = fail(LGS_ERR_HIP, "etab upload: %s", hipGetErrorString(e));
        }
        if (rc) {
            (void)hipStreamDestroy(c->own);
            delete c;
            return rc;
        }
        // Taylor coefficients per grid point (lgs_device.h CoefTab), long double
        std::vector<double> t2((size_t)(lgs::kErfTabLast + 1) * lgs::kCoefStride, 0.0);
        const long double two_over_sqrtpi = 1.128379167095512573896158903121545172L;
        for (int j = 0; j <= lgs::kErfTabLast; ++j) {
            const long double y0 = (long double)j / 64.0L, G = expl(-y0 * y0);
            long double H[10];
            H[0] = 1.0L;
            H[1] = 2.0L * y0;
            for (int m = 1; m < 9; ++m) H[m + 1] = 2.0L * y0 * H[m] - 2.0L * m * H[m - 1];
            double* r = t2.data() + (size_t)j * lgs::kCoefStride;
            r[0] = (double)erfl(y0);
            long double fact = 1.0L;
            for (int m = 1; m <= 7; ++m) {
                fact *= m;
                r[m] = (double)(two_over_sqrtpi * ((m - 1) % 2 ? -1.0L : 1.0L) * H[m - 1] * G / fact);
            }
            fact = 1.0L;
            for (int m = 0; m <= 8; ++m) {
                if (m) fact *= m;
                r[8 + m] = (double)((m % 2 ? -1.0L : 1.0L) * H[m] * G / fact);
            }
        }
        rc = c->etab2.reserve(t2.size() * 8);
        if (!rc) {
            e = hipMemcpy(c->etab2.p, t2.data(), t2.size() * 8, hipMemcpyHostToDevice);
            if (e != hipSuccess) rc = fail(LGS_ERR_HIP, "etab2 upload: %s", hipGetErrorString(e));
        }
        if (rc) {
            (void)hipStreamDestroy(c->own);
            delete c;
            return rc;
        }
    }
    *out = c;
    return LGS_OK;
}

int lgs_destroy(lgs_ctx* c) {
    if (!c) return LGS_OK;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto& t : c->pending) {
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
    for (auto e : c->pool) (void)hipEventDestroy(e);
    if (c->fw_ev) (void)hipEventDestroy(c->fw_ev);
    if (c->fw_host) (void)hipHostFree(c->fw_host);
    for (hipStream_t ks : {c->kstream_full, c->kstream_split})
        if (ks) {
            (void)hipStreamSynchronize(ks);
            (void)hipStreamDestroy(ks);
        }
    if (c->kt0) (void)hipEventDestroy(c->kt0);
    if (c->kt1) (void)hipEventDestroy(c->kt1);
    if (c->ev_klein) (void)hipEventDestroy(c->ev_klein);
    if (c->spec.ev) (void)hipEventDestroy(c->spec.ev);
    for (auto& s : c->bset)
        if (s.ev_free) (void)hipEventDestroy(s.ev_free);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
    return LGS_OK;
}

int lgs_set_stream(lgs_ctx* c, void* s) {
    int rc = check_ctx(c, false);
    if (rc) return rc;
    const hipStream_t ns = s ? (hipStream_t)s : c->own;
    // the old stream may still run an early-checked lgs_imhk's later launches, which
    // read the context's buffers: finish them before another stream reuses those
    if (ns != c->stream) HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->kstream) HIP_TRY(hipStreamSynchronize(c->kstream));  // (a look-ahead launch stays valid)
    c->stream = ns;
    return LGS_OK;
}


int lgs_set_basis(lgs_ctx* c, int64_t d, const double* R, const double* cprime, const double* B,
                  double sigma, int32_t precision, uint32_t flags) {
    int rc = check_ctx(c, false);
    if (rc) return rc;
    if (d <= 0 || d > (1 << 20)) return fail(LGS_ERR_INVALID, "dimension %lld out of range", (long long)d);
    if (!R || !cprime) return fail(LGS_ERR_INVALID, "R and cprime are required");
    if (!(sigma > 0) || !std::isfinite(sigma))
        return fail(LGS_ERR_INVALID, "Standard deviation must be positive, got %g", sigma);
    if (precision <= 0) return fail(LGS_ERR_INVALID, "precision must be positive");
    // an early-checked lgs_imhk / an asynchronous lgs_gram may still run on the
    // context's stream and read R, BT, the digit planes, records, EMAX: the blocking
    // copies below are not ordered after a non-blocking stream's work
    HIP_TRY(hipStreamSynchronize(c->stream));
    if ((rc = spec_discard(c))) return rc;  // (a look-ahead launch reads the basis being replaced)
    if (c->kstream_split && c->cu_split != 0 && !hook("LGS_PIPE_CU_RESERVE")) {  // the CU split decided anew
        HIP_TRY(hipStreamSynchronize(c->kstream));
        c->kstream = c->kstream_full;
        c->kstream_cus = 0;
        c->cu_split = 0;
    }
    c->kt_pending = false;
    const int PB = c->panel;
    const size_t dd = (size_t)d;
    // per-coordinate parameters (klein.py:195-211, 255-263)
    std::vector<double> co(8 * dd);
    for (size_t i = 0; i < dd; ++i) {
        const double rii = R[i * dd + i];
        if (rii == 0.0 || !std::isfinite(rii))
            return fail(LGS_ERR_INVALID, "R[%zu,%zu] must be finite and non-zero", i, i);
        const double sref = sigma / std::fabs(rii);
        double s = sref;
        if (sref < 1e-10)
            s = 0.0;  // deterministic rounding
        else if (sref > 1e10)
            s = std::min(sref, 1e6);
        co[i] = cprime[i];
        co[dd + i] = rii;
        co[2 * dd + i] = s;
        co[3 * dd + i] = sref;
        co[4 * dd + i] = 0.5 * std::log(2.0 * M_PI) + std::log(sref);
        co[5 * dd + i] = 1.0 / rii;
        co[6 * dd + i] = rii / sigma;
        co[7 * dd + i] = 1.0 / sref;
    }
    std::vector<double> szc(dd * lgs::kSzcStride);
    for (size_t i = 0; i < dd; ++i) lgs_host::build_szc(co[2 * dd + i], precision, szc.data() + i * lgs::kSzcStride);
    // Decision certificate of the blocked kernels (lgs_device.h "certified
    // decisions"): |mu_fast - mu_ref| <= Ca + Cb * sum_{j>i} |z_j| + 6e-16 |mu|, with
    // M = max_{j>i} |R_ij|, L1 = sum_{j>i} |R_ij|, u = 2^-53:
    //  * both sums of R_ij z_j against the exact one: the reference's sequential sum
    //    gamma_d, the blocked FMA / MFMA sums gamma_{d+40}  -> (2d+80) 1.1 u M Z1;
    //  * int8-digit far field: R rounded to 2^(E-8D) with D = kOzDigits, at most
    //    2^(E-8D-1) <= 2^(2-8D) M = 2^(55-8D) u M per unit of z (u M / 2 at D = 7,
    //    128 u M at D = 6), and the recombination of the D + 1 digit classes, D <= 7
    //    roundings of at most sum_j (|R_ij| + 2^E/256)(|z_j| + 512) with 2^E <= 8 M
    //    -> (2 + 2^(55-8D)) u M Z1 in Cb, 7.1 u (512 L1 + 16 M d) in Ca;
    //  * subtraction, reciprocal / division: 5 u |mu| (the kernels' 6e-16 |mu|).
    std::vector<double> cert(2 * dd, 0.0), cbc(dd, 0.0);
    {
        const double u = 0x1p-53, g = (2.0 * (double)d + 80.0) * u;
        for (size_t i = 0; i < dd; ++i) {
            double M = 0.0, L1 = 0.0;
            for (size_t j = i + 1; j < dd; ++j) {
                const double r = std::fabs(R[i * dd + j]);
                M = std::max(M, r);
                L1 += r;
            }
            const double ir = 1.0 / std::fabs(R[i * dd + i]);
            const double ca = 1.01 * 7.1 * u * (512.0 * L1 + 16.0 * M * (double)d) * ir;
            const double cb = 1.01 * (1.1 * g / (1.0 - g) + (2.0 + std::ldexp(1.0, 55 - 8 * lgs::kOzDigits)) * u) * M * ir;
            cert[2 * i] = ca;
            cert[2 * i + 1] = cb;
            // coarse far field (klein_mfma_kernel, reference mode, panels of two
            // speculative sub-panels): the digits below the kOzCoarse most significant
            // ones are dropped, |dropped| <= 128 (256^-4 + 256^-5 + 256^-6) 2^E
            // < 2^(E - 24.99) <= 2^(31.01) u M per unit of z, plus the rounding above
            cbc[i] = 1.01 * (1.1 * g / (1.0 - g) + (2.0 + std::ldexp(1.0, 55 - 8 * lgs::kOzDigits) +
                                                    std::ldexp(1.0, 56 - 8 * lgs::kOzCoarse)) * u) * M * ir;
            szc[i * lgs::kSzcStride + lgs::kSzCa] = ca;
            szc[i * lgs::kSzcStride + lgs::kSzCb] = cb;
        }
    }
    // initial cap on sum_j |z_j| (32-row-panel kernels): window half-widths with room
    // for the conditional means; replaced by twice the largest sum seen once a launch
    // has reported it (finish)
    c->z1seen = 0.0;
    c->z1cap = 0.0;
    for (size_t i = 0; i < dd; ++i) c->z1cap += 16.0 * co[2 * dd + i] + 4.0;
    if (hook("LGS_DEBUG_SZC")) {
        int hist[5] = {0, 0, 0, 0, 0};
        for (size_t i = 0; i < dd; ++i) hist[(int)szc[i * lgs::kSzcStride + 2]]++;
        fprintf(stderr, "lgs: SampleZ kinds round %d small %d closed %d capped %d generic %d\n", hist[0],
                hist[1], hist[2], hist[3], hist[4]);
    }
    // panel layouts (lgs_kernels.hip, klein_panel_kernel)
    const int64_t npan = (d + PB - 1) / PB;
    size_t rp_elems = (size_t)PB * PB * (size_t)(npan * (npan - 1) / 2);
    std::vector<double> rp(std::max<size_t>(rp_elems, 1), 0.0);
    for (int64_t pk = 0; pk < npan; ++pk) {
        const int64_t p_hi = d - pk * PB;
        const size_t off = (size_t)PB * PB * (size_t)(pk * (pk - 1) / 2);
        for (int64_t j = p_hi; j < d; ++j)
            for (int r = 0; r < PB; ++r) {
                const int64_t row = p_hi - PB + r;
                rp[off + (size_t)(j - p_hi) * PB + r] = row >= 0 ? R[(size_t)row * dd + j] : 0.0;
            }
    }
    std::vector<double> rcv(dd * (PB - 1), 0.0);
    for (int64_t i = 0; i < d; ++i) {
        const int64_t pk = (d - 1 - i) / PB;
        const int64_t p_lo = std::max<int64_t>(0, d - (pk + 1) * PB);
        for (int m = 0; m < PB - 1; ++m) {
            const int64_t row = i - 1 - m;
            rcv[(size_t)i * (PB - 1) + m] = row >= p_lo ? R[(size_t)row * dd + i] : 0.0;
        }
    }
    // 32-row panels, two-level near field (klein_mfma_kernel): RS = near-field
    // columns of 16-row sub-panels, RX = per panel the block R[p_hi-32+nq][p_hi-16+4kk+kq]
    // in MFMA A-fragment order [kk][lane = 16 kq + nq] (0 for rows < 0)
    std::vector<double> rsv(dd * 15, 0.0), rxv;
    for (int64_t i = 0; i < d; ++i) {
        const int64_t sp = (d - 1 - i) / 16;
        const int64_t s_lo = std::max<int64_t>(0, d - (sp + 1) * 16);
        for (int m = 0; m < 15; ++m) {
            const int64_t row = i - 1 - m;
            rsv[(size_t)i * 15 + m] = row >= s_lo ? R[(size_t)row * dd + i] : 0.0;
        }
    }
    rxv.assign((size_t)256 * ((d + 31) / 32), 0.0);
    for (int64_t pk = 0; pk < (d + 31) / 32; ++pk) {
        const int64_t p_hi = d - 32 * pk;
        for (int kk = 0; kk < 4; ++kk)
            for (int l = 0; l < 64; ++l) {
                const int64_t row = p_hi - 32 + (l & 15), col = p_hi - 16 + 4 * kk + (l >> 4);
                if (row >= 0 && col >= 0 && col < d)
                    rxv[(size_t)pk * 256 + kk * 64 + l] = R[(size_t)row * dd + col];
            }
    }
    // int8-digit far field (klein_mfma_kernel OZ): per 32-row panel, rows scaled by
    // 2^E_i (|R_ij| 2^-E_i < 1/4 over the panel's far columns j >= p_hi), rounded
    // to 2^(E_i - 8 kOzDigits) and split into kOzDigits balanced base-256 digits.
    const int64_t npan32 = (d + 31) / 32;
    std::vector<double> rscale(dd, 1.0);
    std::vector<int64_t> rdoff(npan32 + 1, 0);
    std::vector<int8_t> rdv;
    bool oz = d <= lgs::kOzMaxD;
    for (size_t k = 0; k < dd * dd && oz; ++k) oz = std::isfinite(R[k]);
    if (oz) {
        for (int64_t pk = 1; pk < npan32; ++pk)
            rdoff[pk + 1] = rdoff[pk] + ((32 * pk + 63) / 64) * 2 * lgs::kOzDigits * 1024;
        rdoff[1] = 0;
        rdv.assign((size_t)std::max<int64_t>(rdoff[npan32], 16), 0);
        for (int64_t pk = 1; pk < npan32; ++pk) {
            const int64_t p_hi = d - 32 * pk, K = d - p_hi, nch = (K + 63) / 64;
            int8_t* base = rdv.data() + rdoff[pk];
            for (int r = 0; r < 32; ++r) {
                const int64_t row = p_hi - 32 + r;
                if (row < 0) continue;
                double mx = 0.0;
                for (int64_t j = p_hi; j < d; ++j) mx = std::max(mx, std::fabs(R[(size_t)row * dd + j]));
                const int E = mx > 0.0 ? std::ilogb(mx) + 3 : 0;
                rscale[row] = std::ldexp(1.0, E);
                const int t = r >> 4, n = r & 15;
                for (int64_t j = p_hi; j < d; ++j) {
                    long long M = std::llrint(std::ldexp(R[(size_t)row * dd + j], 8 * lgs::kOzDigits - E));
                    const int64_t kk = j - p_hi, ch = kk / 64, h = (kk % 64) / 16, e = kk % 16;
                    for (int a = lgs::kOzDigits; a >= 1; --a) {  // least significant digit first
                        const long long dg = ((M % 256) + 256 + 128) % 256 - 128;
                        M = (M - dg) / 256;
                        const int64_t lane = h * 16 + n;
                        base[(((ch * 2 + t) * lgs::kOzDigits + (a - 1)) * 64 + lane) * 16 + e] = (int8_t)dg;
                    }
                    if (M != 0) return fail(LGS_ERR_INVALID, "R digit split overflow");
                }
            }
            (void)nch;
        }
    }
    // per-coordinate records (lgs_kernels.h kRec*)
    std::vector<double> crec(dd * lgs::kRecStride, 0.0);
    for (size_t i = 0; i < dd; ++i) {
        double* r = crec.data() + i * lgs::kRecStride;
        std::copy(szc.data() + i * lgs::kSzcStride, szc.data() + i * lgs::kSzcStride + lgs::kSzUsed, r);
        r[lgs::kRecCp] = co[i];
        r[lgs::kRecIrii] = co[5 * dd + i];
        r[lgs::kRecRos] = co[6 * dd + i];
        r[lgs::kRecIsr] = co[7 * dd + i];
        r[lgs::kRecLterm] = co[4 * dd + i];
        std::copy(rsv.data() + i * 15, rsv.data() + i * 15 + 15, r + lgs::kRecRs);
        r[lgs::kRecScale] = rscale[i];
        r[lgs::kRecCbC] = cbc[i];
        const int kind = (int)r[2];
        r[lgs::kRecDisp] = r[0] != 0.0 && kind == lgs::kSzSmall && r[7] == 0.0   ? 0.0
                           : r[0] != 0.0 && kind == lgs::kSzCapped && r[7] == 1.0 ? 1.0
                                                                                    : 2.0;
    }
    for (int64_t top = d; top >= 16; top -= 16) {  // whole 16-row sub-panels (top = d - 16 sp)
        bool all = true;
        for (int64_t i = top - 16; i < top && all; ++i) {
            const double* r = crec.data() + i * lgs::kRecStride;
            all = r[0] != 0.0 && (int)r[2] == lgs::kSzSmall && r[7] == 0.0;
        }
        for (int64_t i = top - 16; i < top; ++i) crec[i * lgs::kRecStride + lgs::kRecSpec] = all ? 1.0 : 0.0;
        if (all) continue;
        // 2: every coordinate of the sub-panel capped with sigma >= 360 (the near field
        // then skips the per-coordinate kind dispatch, klein_mfma_kernel)
        bool cap = true;
        for (int64_t i = top - 16; i < top && cap; ++i) {
            const double* r = crec.data() + i * lgs::kRecStride;
            cap = r[0] != 0.0 && (int)r[2] == lgs::kSzCapped && r[7] == 1.0;
        }
        if (cap)
            for (int64_t i = top - 16; i < top; ++i) crec[i * lgs::kRecStride + lgs::kRecSpec] = 2.0;
    }
    // q-panel skip (klein_mfma_kernel, reference mode): for a 32-row panel whose rows
    // all lie in speculative sub-panels, the largest ||z_W||_2^2 (W = coordinates
    // outside speculative sub-panels; the kernel tracks it per sample while every
    // speculative z so far is 0) for which every row i is certified z_i = 0 without
    // its mean: the reference's mean obeys
    //   |mu_i| <= (|c'_i| + (1 + g) sum_j |R_ij z_j|) (1 + 3u) / R_ii,
    //   sum_j |R_ij z_j| <= G_i ||z_W||,  G_i = ||R[i, j > i, j in W]||_2  (Cauchy-Schwarz),
    // g = 1.1 d u (the sum's rounding), and the one-dominant-point decision z = rint(mu)
    // = 0 holds for every |mu| < theta_i = 1/2 - 745.2 / (is_i^2 (1 - 1e-12)) (all other
    // window points below e^-745.2, lgs_device.h; q[7] == 0: the window ends carry 0).
    std::vector<double> qz2((size_t)npan32, -1.0);
    bool any_q = false;
    if (!(flags & LGS_BASIS_LINEAR_PROBS)) {
        std::vector<char> inW(dd);
        for (size_t i = 0; i < dd; ++i) inW[i] = crec[i * lgs::kRecStride + lgs::kRecSpec] != 1.0;
        const double g = 1.1 * (double)d * std::ldexp(1.0, -53);
        for (int64_t pk = 0; pk < npan32; ++pk) {
            const int64_t p_hi = d - 32 * pk;
            if (p_hi < 32) break;
            bool all = true;
            for (int64_t i = p_hi - 32; i < p_hi && all; ++i) all = !inW[i];
            if (!all) continue;
            double zmin = INFINITY;
            for (int64_t i = p_hi - 32; i < p_hi; ++i) {
                long double g2 = 0.0L;
                for (int64_t j = i + 1; j < d; ++j)
                    if (inW[j]) g2 += (long double)R[i * dd + j] * (long double)R[i * dd + j];
                const double Gi = (double)sqrtl(g2) * (1.0 + 1e-13);
                const double is = szc[i * lgs::kSzcStride + 1];
                const double theta = 0.5 - 745.2 / (is * is * (1.0 - 1e-12)) - 1e-9;
                const double num = theta * co[dd + i] * (1.0 - 1e-12) - std::fabs(co[i]);
                const double zi = num <= 0.0 ? -1.0 : (Gi > 0.0 ? num / ((1.0 + g) * Gi) : INFINITY);
                zmin = std::min(zmin, zi);
            }
            if (zmin > 0.0) {
                qz2[pk] = std::isinf(zmin) ? INFINITY : zmin * zmin * (1.0 - 1e-12);
                any_q = true;
            }
        }
    }
    c->has_qz2 = any_q;
    if (any_q) {
        if ((rc = c->QZ2.reserve(qz2.size() * 8))) return rc;
        HIP_TRY(hipMemcpy(c->QZ2.p, qz2.data(), qz2.size() * 8, hipMemcpyHostToDevice));
    }
    c->has_rd = oz;
    if (oz) {
        if ((rc = c->RD.reserve(rdv.size())) || (rc = c->RDOFF.reserve(rdoff.size() * 8))) return rc;
        HIP_TRY(hipMemcpy(c->RD.p, rdv.data(), rdv.size(), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->RDOFF.p, rdoff.data(), rdoff.size() * 8, hipMemcpyHostToDevice));
    }
    if ((rc = c->CREC.reserve(crec.size() * 8)) || (rc = c->RX.reserve(rxv.size() * 8))) return rc;
    HIP_TRY(hipMemcpy(c->CREC.p, crec.data(), crec.size() * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->RX.p, rxv.data(), rxv.size() * 8, hipMemcpyHostToDevice));
    if ((rc = c->R.reserve(dd * dd * 8)) || (rc = c->RP.reserve(rp.size() * 8)) ||
        (rc = c->RC.reserve(rcv.size() * 8)) || (rc = c->coord.reserve(co.size() * 8)) ||
        (rc = c->szc.reserve(szc.size() * 8)) || (rc = c->CERT.reserve(cert.size() * 8)))
        return rc;
    HIP_TRY(hipMemcpy(c->CERT.p, cert.data(), cert.size() * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->szc.p, szc.data(), szc.size() * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->R.p, R, dd * dd * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->RP.p, rp.data(), rp.size() * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->RC.p, rcv.data(), rcv.size() * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->coord.p, co.data(), co.size() * 8, hipMemcpyHostToDevice));
    {  // R transposed (certified Wang-Ling accept decisions: reference-order means, coalesced)
        std::vector<double> rt(dd * dd);
        for (size_t r = 0; r < dd; ++r)
            for (size_t k = 0; k < dd; ++k) rt[k * dd + r] = R[r * dd + k];
        if ((rc = c->RT.reserve(dd * dd * 8)) || (rc = c->EMAX.reserve(8))) return rc;
        HIP_TRY(hipMemcpy(c->RT.p, rt.data(), dd * dd * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemset(c->EMAX.p, 0, 8));
    }
    c->has_B = B != nullptr;
    if (B) {
        std::vector<double> bt(dd * dd);
        for (size_t r = 0; r < dd; ++r)
            for (size_t k = 0; k < dd; ++k) bt[k * dd + r] = B[r * dd + k];
        if ((rc = c->BT.reserve(dd * dd * 8))) return rc;
        HIP_TRY(hipMemcpy(c->BT.p, bt.data(), dd * dd * 8, hipMemcpyHostToDevice));
        // exact int8-digit planes when B is integral with |B| <= 32639
        bool ok = true;
        for (size_t k = 0; k < dd * dd && ok; ++k)
            ok = B[k] == std::nearbyint(B[k]) && std::fabs(B[k]) <= 32639.0;
        c->has_Bi8 = ok;
        if (ok) {
            const int64_t rows = (d + 127) / 128 * 128, cols = (d + 63) / 64 * 64;
            std::vector<int8_t> planes((size_t)2 * rows * cols, 0);
            int8_t* hi = planes.data();
            int8_t* lo = hi + (size_t)rows * cols;
            for (size_t r = 0; r < dd; ++r)
                for (size_t k = 0; k < dd; ++k) {
                    const int v = (int)B[r * dd + k];
                    const int l = (v << 24) >> 24;
                    hi[r * cols + k] = (int8_t)((v - l) >> 8);
                    lo[r * cols + k] = (int8_t)l;
                }
            if ((rc = c->Bd.reserve(planes.size()))) return rc;
            HIP_TRY(hipMemcpy(c->Bd.p, planes.data(), planes.size(), hipMemcpyHostToDevice));
            // block sparsity of B for bz_i8_kernel: an all-zero 128 x 64 block contributes
            // exactly nothing, so its K chunk is skipped (NTRU [[qI,0],[H,I]]: 62% of blocks)
            // (bit 16 of an entry: the first row tile listing the chunk owns its share of
            // the kept states' moments when B z computes them, bz_i8_kernel MP; B has full
            // rank, so every chunk has an owner)
            std::vector<int> kc, ko(1, 0);
            std::vector<char> owned((size_t)(cols / 64), 0);
            for (int64_t rt = 0; rt < rows / 128; ++rt) {
                for (int64_t ch = 0; ch < cols / 64; ++ch) {
                    bool nz = false;
                    for (int64_t r = rt * 128; r < rt * 128 + 128 && !nz; ++r)
                        for (int64_t k = ch * 64; k < ch * 64 + 64 && !nz; ++k)
                            nz = hi[r * cols + k] != 0 || lo[r * cols + k] != 0;
                    if (nz) {
                        kc.push_back((int)ch | (owned[ch] ? 0 : 1 << 16));
                        owned[ch] = 1;
                    }
                }
                ko.push_back((int)kc.size());
            }
            if (kc.empty()) kc.push_back(0);
            c->bz_mom_ok = std::all_of(owned.begin(), owned.end(), [](char o) { return o != 0; });
            if ((rc = c->kchunk.reserve(kc.size() * 4)) || (rc = c->koff.reserve(ko.size() * 4))) return rc;
            HIP_TRY(hipMemcpy(c->kchunk.p, kc.data(), kc.size() * 4, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(c->koff.p, ko.data(), ko.size() * 4, hipMemcpyHostToDevice));
            c->bd_rows = rows;
            c->bd_cols = cols;
        }
    } else {
        c->has_Bi8 = false;
    }
    c->d = d;
    c->sigma = sigma;
    c->precision = precision;
    c->basis_flags = flags;
    // proposals per launch: the coefficient store up to 32 GiB (288 GB of HBM; a
    // pipelined lgs_imhk holds two such sets) and 2^22 proposals (round 5: a 2^21-
    // proposal block runs the C3 bench at 110 vs 105 M samples/s -- the launch's tail
    // and the per-block work amortised, profiles/r05aa_bench_ab.log)
    const int64_t cap = std::max<int64_t>(256, (int64_t)((size_t)32 << 30) / (8 * d));
    if (!c->max_props_user) c->max_props = std::min<int64_t>(std::max<int64_t>(cap, 256), 1 << 22);
    return LGS_OK;
}

int lgs_klein(lgs_ctx* c, uint64_t seed, uint64_t first, int64_t n, void* z_out, double* v_out,
              double* logw_out, uint32_t flags) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (n < 0) return fail(LGS_ERR_INVALID, "n < 0");
    if (n == 0) return LGS_OK;
    const bool dev = flags & LGS_DEVICE_PTRS, z64 = flags & LGS_Z64,
               cm = flags & LGS_COORD_MAJOR, exact = flags & LGS_EXACT_ORDER,
               wl = flags & LGS_WANG_LING, bound = flags & LGS_LOGW_BOUND;
    if (v_out && !c->has_B) return fail(LGS_ERR_STATE, "v_out requires B");
    const int64_t d = c->d;
    const int ob = z64 ? 8 : 4;  // caller's coefficient width
    if ((rc = reset_flags(c))) return rc;
    const int64_t chunk = std::min<int64_t>(n, c->max_props);
    // direct device coordinate-major output: the kernel writes straight into z_out;
    // otherwise an internal store (16-bit unless int64 / coordinate-major output)
    const bool direct = dev && cm && z_out;
    int zb = (direct || ob == 8 || (z_out && cm)) ? ob : c->zint;
    if (!direct && (rc = c->Z.reserve((size_t)chunk * d * std::max(zb, 4)))) return rc;
    if ((rc = c->LW.reserve((size_t)chunk * 8))) return rc;
    if (!dev) {
        if (z_out && (rc = c->stage_a.reserve((size_t)chunk * d * ob))) return rc;
        if (v_out && (rc = c->V.reserve((size_t)chunk * d * 8))) return rc;
    }
    for (int64_t off = 0; off < n; off += chunk) {
        const int64_t m = std::min<int64_t>(chunk, n - off);
        lgs::KleinArgs a = base_args(c, seed);
        a.counter_mode = 0;
        a.base = first + (uint64_t)off;
        a.n = m;
        void* Zp;
        if (direct) {
            Zp = (char*)z_out + (size_t)off * ob;
            a.ldz = n;
        } else {
            Zp = c->Z.p;
            a.ldz = m;
        }
        a.LW = logw_out ? (dev ? logw_out + off : c->LW.as<double>()) : nullptr;
        if (wl && !exact) a.emax = c->EMAX.as<unsigned long long>();
        if (wl && bound && logw_out) {  // the weights' bounds into logw_out[n .. 2n)
            if (dev) {
                a.LWE = logw_out + n + off;
            } else {
                if ((rc = c->LWE.reserve((size_t)chunk * 8))) return rc;
                a.LWE = c->LWE.as<double>();
            }
        }
        if ((rc = run_klein_store(c, a, exact, wl, zb, Zp, false))) return rc;
        if (z_out && !direct) {
            if (cm) {  // coordinate-major output through host pointers (zb == ob)
                for (int64_t i = 0; i < d; ++i)
                    HIP_TRY(hipMemcpy2DAsync((char*)z_out + ((size_t)i * n + off) * ob, 0,
                                             (char*)Zp + (size_t)i * m * ob, 0, m * ob, 1,
                                             kind_of(dev, true), c->stream));
            } else {
                void* dst = dev ? (char*)z_out + (size_t)off * d * ob : c->stage_a.p;
                HIP_TRY(lgs::launch::transpose_out(Zp, zb, a.ldz, m, (int)d, dst, ob, c->stream));
                if (!dev)
                    HIP_TRY(hipMemcpyAsync((char*)z_out + (size_t)off * d * ob, dst, (size_t)m * d * ob,
                                           hipMemcpyDeviceToHost, c->stream));
            }
        }
        if (v_out) {
            double* V = dev ? v_out + (size_t)off * d : c->V.as<double>();
            if ((rc = run_bz(c, Zp, zb, a.ldz, m, V, 0, 0, 0, nullptr, true))) return rc;
            if ((rc = settle_bz(c))) return rc;
            if (!dev)
                HIP_TRY(hipMemcpyAsync(v_out + (size_t)off * d, V, (size_t)m * d * 8,
                                       hipMemcpyDeviceToHost, c->stream));
        }
        if (logw_out && !dev)
            HIP_TRY(hipMemcpyAsync(logw_out + off, a.LW, (size_t)m * 8, hipMemcpyDeviceToHost,
                                   c->stream));
        if (logw_out && !dev && a.LWE)
            HIP_TRY(hipMemcpyAsync(logw_out + n + off, a.LWE, (size_t)m * 8, hipMemcpyDeviceToHost,
                                   c->stream));
        if (!dev || v_out) {  // staging buffers / the int8-digit replay need the chunk intact
            if ((rc = finish(c))) return rc;
        }
    }
    return finish(c);
}

int lgs_lattice_points(lgs_ctx* c, int64_t n, const void* z, double* v_out, uint32_t flags) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (n <= 0) return n == 0 ? LGS_OK : fail(LGS_ERR_INVALID, "n < 0");
    if (!z || !v_out) return fail(LGS_ERR_INVALID, "null buffer");
    const bool dev = flags & LGS_DEVICE_PTRS, z64 = flags & LGS_Z64, cm = flags & LGS_COORD_MAJOR;
    const int64_t d = c->d;
    const int zb = z64 ? 8 : 4;
    if ((rc = reset_flags(c))) return rc;
    const void* Zc = z;
    if (!dev || !cm) {
        if ((rc = c->Z.reserve((size_t)n * d * zb)) || (rc = c->stage_a.reserve((size_t)n * d * zb)))
            return rc;
        const void* src = z;
        if (!dev) {
            HIP_TRY(hipMemcpyAsync(c->stage_a.p, z, (size_t)n * d * zb, hipMemcpyHostToDevice, c->stream));
            src = c->stage_a.p;
        }
        if (cm) {
            Zc = src;
        } else {
            HIP_TRY(lgs::launch::to_coord_major(src, zb, n, (int)d, c->Z.p, zb, n, c->stream));
            Zc = c->Z.p;
        }
    }
    double* V = v_out;
    if (!dev) {
        if ((rc = c->V.reserve((size_t)n * d * 8))) return rc;
        V = c->V.as<double>();
    }
    if ((rc = run_bz(c, Zc, zb, n, n, V))) return rc;
    if ((rc = settle_bz(c))) return rc;
    if (!dev) HIP_TRY(hipMemcpyAsync(v_out, V, (size_t)n * d * 8, hipMemcpyDeviceToHost, c->stream));
    return finish(c);
}

int lgs_log_density(lgs_ctx* c, int64_t n, const void* z, double* out, uint32_t flags) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (n <= 0) return n == 0 ? LGS_OK : fail(LGS_ERR_INVALID, "n < 0");
    if (!z || !out) return fail(LGS_ERR_INVALID, "null buffer");
    const bool dev = flags & LGS_DEVICE_PTRS, z64 = flags & LGS_Z64, cm = flags & LGS_COORD_MAJOR;
    const int64_t d = c->d;
    const int zb = z64 ? 8 : 4;
    if ((rc = reset_flags(c))) return rc;
    const void* Zc = z;
    if (!dev || !cm) {
        if ((rc = c->Z.reserve((size_t)n * d * zb)) || (rc = c->stage_a.reserve((size_t)n * d * zb)))
            return rc;
        const void* src = z;
        if (!dev) {
            HIP_TRY(hipMemcpyAsync(c->stage_a.p, z, (size_t)n * d * zb, hipMemcpyHostToDevice, c->stream));
            src = c->stage_a.p;
        }
        if (cm) {
            Zc = src;
        } else {
            HIP_TRY(lgs::launch::to_coord_major(src, zb, n, (int)d, c->Z.p, zb, n, c->stream));
            Zc = c->Z.p;
        }
    }
    double* o = out;
    if (!dev) {
        if ((rc = c->LW.reserve((size_t)n * 8))) return rc;
        o = c->LW.as<double>();
    }
    lgs::KleinArgs a = base_args(c, 0);
    a.n = n;
    a.ldz = n;
    HIP_TRY(lgs::launch::log_density(a, c->R.as<double>(), Zc, zb, o, c->stream));
    if (!dev) HIP_TRY(hipMemcpyAsync(out, o, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
    return finish(c);
}

static int imhk_impl(lgs_ctx* c, uint64_t seed, uint64_t first_chain, int64_t nc, uint64_t first_step,
                     int64_t n_steps, int32_t thin, void* z_state, double* logw_state, int32_t* state_init,
                     int64_t* accepts, void* z_samples, double* v_samples, int64_t* moments,
                     double* logw_samples, uint8_t* accepted, double* vnorm2_samples, int64_t* zk_samples,
                     int64_t zk_index, int64_t fn_chains, const lgs_imhk_outputs* lag, uint32_t flags);

int lgs_imhk(lgs_ctx* c, uint64_t seed, uint64_t first_chain, int64_t nc, uint64_t first_step,
             int64_t n_steps, int32_t thin, void* z_state, double* logw_state, int32_t* state_init,
             int64_t* accepts, void* z_samples, double* v_samples, int64_t* moments,
             uint32_t flags) {
    return imhk_impl(c, seed, first_chain, nc, first_step, n_steps, thin, z_state, logw_state, state_init,
                     accepts, z_samples, v_samples, moments, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr, flags);
}

int lgs_imhk_trace(lgs_ctx* c, uint64_t seed, uint64_t first_chain, int64_t nc, uint64_t first_step,
                   int64_t n_steps, int32_t thin, void* z_state, double* logw_state, int32_t* state_init,
                   int64_t* accepts, void* z_samples, double* v_samples, int64_t* moments,
                   double* logw_samples, uint8_t* accepted, uint32_t flags) {
    return imhk_impl(c, seed, first_chain, nc, first_step, n_steps, thin, z_state, logw_state, state_init,
                     accepts, z_samples, v_samples, moments, logw_samples, accepted, nullptr, nullptr, 0, 0, nullptr, flags);
}

int lgs_imhk_ex(lgs_ctx* c, uint64_t seed, uint64_t first_chain, int64_t nc, uint64_t first_step,
                int64_t n_steps, int32_t thin, void* z_state, double* logw_state, int32_t* state_init,
                int64_t* accepts, void* z_samples, double* v_samples, int64_t* moments,
                const lgs_imhk_outputs* out, uint32_t flags) {
    if (!out)
        return imhk_impl(c, seed, first_chain, nc, first_step, n_steps, thin, z_state, logw_state, state_init,
                         accepts, z_samples, v_samples, moments, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr, flags);
    return imhk_impl(c, seed, first_chain, nc, first_step, n_steps, thin, z_state, logw_state, state_init,
                     accepts, z_samples, v_samples, moments, out->logw_samples, out->accepted,
                     out->vnorm2_samples, out->zk_samples, out->zk_index, out->fn_chains,
                     out->lag_L > 0 ? out : nullptr, flags);
}

static int imhk_impl(lgs_ctx* c, uint64_t seed, uint64_t first_chain, int64_t nc, uint64_t first_step,
                     int64_t n_steps, int32_t thin, void* z_state, double* logw_state, int32_t* state_init,
                     int64_t* accepts, void* z_samples, double* v_samples, int64_t* moments,
                     double* logw_samples, uint8_t* accepted, double* vnorm2_samples, int64_t* zk_samples,
                     int64_t zk_index, int64_t fn_chains, const lgs_imhk_outputs* lag, uint32_t flags) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (nc < 0 || n_steps < 0 || thin < 1) return fail(LGS_ERR_INVALID, "bad nc/n_steps/thin");
    if (first_step < 1) return fail(LGS_ERR_INVALID, "first_step must be >= 1 (step 0 is the initial draw)");
    if (!z_state || !logw_state || !state_init || !accepts)
        return fail(LGS_ERR_INVALID, "z_state, logw_state, state_init and accepts are required");
    const bool dev = flags & LGS_DEVICE_PTRS, z64 = flags & LGS_Z64,
               cm = flags & LGS_COORD_MAJOR, exact = flags & LGS_EXACT_ORDER,
               wl = flags & LGS_WANG_LING;
    if (v_samples && !c->has_B) return fail(LGS_ERR_STATE, "v_samples requires B");
    if (v_samples && !dev)
        return fail(LGS_ERR_INVALID, "v_samples needs LGS_DEVICE_PTRS (use lgs_lattice_points on z_samples)");
    if (z_samples && cm)
        return fail(LGS_ERR_INVALID, "z_samples is row-major (n_chains x n_keep x d) only");
    if ((vnorm2_samples || zk_samples) && !dev)
        return fail(LGS_ERR_INVALID, "vnorm2_samples / zk_samples need LGS_DEVICE_PTRS");
    if (vnorm2_samples && !v_samples) return fail(LGS_ERR_INVALID, "vnorm2_samples needs v_samples");
    if (zk_samples && (zk_index < 0 || zk_index >= c->d)) return fail(LGS_ERR_INVALID, "zk_index out of range");
    if (fn_chains < 0 || fn_chains > nc) return fail(LGS_ERR_INVALID, "fn_chains must be in [0, n_chains]");
    if (fn_chains == 0) fn_chains = nc;  // the functionals of every chain's kept states
    if (lag) {
        if (lag->lag_L > (1 << 20)) return fail(LGS_ERR_INVALID, "lag_L too large");
        if ((lag->lag_z_sums && (!zk_samples || !lag->lag_z_ring)) ||
            (lag->lag_v_sums && (!vnorm2_samples || !lag->lag_v_ring)))
            return fail(LGS_ERR_INVALID, "lag sums need their series (zk_samples / vnorm2_samples) and ring");
    }
    if (nc == 0) return LGS_OK;
    if (first_chain + (uint64_t)nc > (1ull << 32) || first_step + (uint64_t)n_steps > (1ull << 32))
        return fail(LGS_ERR_INVALID, "chain / step counters must stay below 2^32");
    const int64_t d = c->d;
    const int ob = z64 ? 8 : 4;      // caller's coefficient width (z_state, z_samples)
    int zb = z64 ? 8 : c->zint;      // internal proposal store width
    const int64_t n_keep = n_steps / thin;
    if ((rc = reset_flags(c))) return rc;
    // Wang-Ling weights of the blocked kernels carry a bounded error: certify each
    // accept decision against it (LGS_EXACT_ORDER weights are the reference's)
    const bool certw = wl && !exact;
    // Early check (device pointers on a caller's stream -- lgs_set_stream orders the
    // caller's work after ours): each block waits only for its abort producers' flag
    // words, not for its accept / moments / B z / gathers, so the caller's next work
    // is enqueued while those run.  Not with the certified Wang-Ling accept (its
    // counters come from the accept kernel).  Timers of the later launches are folded
    // once they finish (fold_timers).  LGS_NO_EARLY_CHECK=1: A/B.
    static const bool no_early = hook_is("LGS_NO_EARLY_CHECK", 1);
    const bool early = dev && c->stream != c->own && !certw && !no_early;
    if (early && !c->fw_host) {
        HIP_TRY(hipHostMalloc((void**)&c->fw_host, 4 * lgs::kFlagWords, hipHostMallocDefault));
        HIP_TRY(hipEventCreateWithFlags(&c->fw_ev, hipEventDisableTiming));
    }

    // proposal store: np columns, plus nc columns for the chain states carried into a
    // block when lattice points are requested (kept-state selections become plain columns)
    const bool carry = v_samples != nullptr;
    // pipelined blocks (see lgs_ctx::BlockSet): the context's own store then only takes
    // the initial draws (nc columns); LGS_CTX_NO_PIPELINE: A/B
    const bool no_pipe = c->no_pipe || hook_is("LGS_NO_PIPE", 1);
    const bool pipe = early && !no_pipe && n_steps > 0;
    if (pipe) {
        if (!c->kstream) {
            // LGS_PIPE_PRIO=1: at the device's highest priority, so the Klein launch's
            // workgroups are dispatched first (measured: no gain, 102.3-102.4 vs
            // 102.6-102.9 M samples/s at the default priority, profiles/r05k_*);
            // 2: at the lowest, so the previous block's dependants go first
            static const int prio = hook("LGS_PIPE_PRIO") ? atoi(hook("LGS_PIPE_PRIO")) : 0;
            // CU split (default; LGS_CTX_NO_CU_SPLIT turns it off): a second Klein stream
            // whose queue is masked off 1/8 of the CUs, so the previous block's
            // store-bound B z finds CUs beside the Klein launch, which otherwise fills
            // every CU's VGPRs and LDS (B z then runs behind it, ~3 % overlap).  Mask bit
            // i is a CU of XCD i % 8 and shader engine (i / 8) % 4, so the top ncu / 8
            // bits take one CU from every shader engine -- an even cut, which the per-SE
            // round-robin workgroup dispatch needs (uneven masks run at the pace of the
            // smallest SE: 16 or 48 spread bits 2x / 1.3x slower,
            // profiles/r06ba_bench_cumask.log; 1/16, 3/32 or 5/32 of the CUs at the top
            // less or slower, r06bb_*).  Which stream is used is decided after the
            // first pipelined call (split_decide).
            // (hooks build: LGS_PIPE_CU_RESERVE=k forces the split with the top k bits,
            // 0 = never; LGS_PIPE_CU_PAT=0 k bits spread over the index space instead)
            const char* h_res = hook("LGS_PIPE_CU_RESERVE");
            static const int cu_pat = hook("LGS_PIPE_CU_PAT") ? atoi(hook("LGS_PIPE_CU_PAT")) : 1;
            int plo = 0, phi = 0, ncu = 0;
            if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) ncu = 0;
            const int cu_res = h_res ? atoi(h_res) : (c->no_cu_split || ncu % 32 != 0 ? 0 : ncu / 8);
            if (prio && hipDeviceGetStreamPriorityRange(&plo, &phi) == hipSuccess && phi != plo)
                HIP_TRY(hipStreamCreateWithPriority(&c->kstream_full, hipStreamNonBlocking, prio == 1 ? phi : plo));
            else
                HIP_TRY(hipStreamCreateWithFlags(&c->kstream_full, hipStreamNonBlocking));
            c->kstream = c->kstream_full;
            c->kstream_cus = 0;
            c->cu_split = 2;
            if (cu_res > 0 && cu_res < ncu) {
                std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
                const int stride = std::max(1, ncu / cu_res);
                int off = 0;
                for (int i = 0; i < ncu; ++i) {
                    const bool res = cu_pat == 1 ? i >= ncu - cu_res : (i % stride == stride - 1 && off < cu_res);
                    if (res && cu_pat != 1) ++off;
                    if (!res) mask[i / 32] |= 1u << (i % 32);
                }
                HIP_TRY(hipExtStreamCreateWithCUMask(&c->kstream_split, (uint32_t)mask.size(), mask.data()));
                HIP_TRY(hipEventCreate(&c->kt0));
                HIP_TRY(hipEventCreate(&c->kt1));
                c->split_cus = ncu - cu_res;
                c->cu_split = 0;
                if (h_res) {  // (forced)
                    c->cu_split = 1;
                    c->kstream = c->kstream_split;
                    c->kstream_cus = c->split_cus;
                }
            }
            HIP_TRY(hipEventCreateWithFlags(&c->ev_klein, hipEventDisableTiming));
        }
        if (!c->kstream_sets_fixed) {
            c->nsets = hook_is("LGS_PIPE_SETS", 3) ? 3 : 2;
            c->kstream_sets_fixed = true;
        }
        for (int si = 0; si < c->nsets; ++si) {
            auto& s = c->bset[si];
            if (!s.ev_free) HIP_TRY(hipEventCreateWithFlags(&s.ev_free, hipEventDisableTiming));
            if (!s.flags.p) {
                if ((rc = s.flags.reserve(4 * lgs::kFlagWords))) return rc;
                HIP_TRY(hipMemset(s.flags.p, 0, 4 * lgs::kFlagWords));
            }
        }
    }
    // ---- block of T steps (a multiple of thin) per Klein launch, and the device buffers
    // of one block.  An allocation that fails halves the block (down to thin steps per
    // chain; the smaller cap stays with the context) instead of returning LGS_ERR_NOMEM.
    int64_t T = 1, np = 0, kmax = 1, own_cols = 0;
    for (int64_t maxp = c->max_props;;) {
        T = std::max<int64_t>(1, maxp / nc);
        if (T < n_steps) T = std::max<int64_t>(thin, (T / thin) * thin);
        T = std::min<int64_t>(T, std::max<int64_t>(n_steps, 1));
        np = nc * T;
        kmax = std::max<int64_t>(T / thin, 1);
        own_cols = pipe ? nc : np + (carry ? nc : 0);
        rc = LGS_OK;
        // (a set in use by an earlier call's dependants is never grown here unless the
        // sizes change -- they depend on nc, T and d only -- and hipFree waits for the device)
        for (int si = 0; pipe && !rc && si < c->nsets; ++si) {
            auto& s = c->bset[si];
            if (!(rc = s.Z.reserve((size_t)(np + (carry ? nc : 0)) * d * std::max(zb, 4))) &&
                !(rc = s.LW.reserve((size_t)np * 8)))
                rc = reserve_oz(c, s.H16, s.ZNZ, s.CLIVE, np);
        }
        if (!rc && !(rc = c->Z.reserve((size_t)own_cols * d * std::max(zb, 4))) &&
            !(rc = c->LW.reserve((size_t)(pipe ? nc : np) * 8)) &&
            !(rc = c->sel.reserve((size_t)std::max<int64_t>(nc * kmax, nc) * 8)) &&
            !(rc = c->fsel.reserve((size_t)nc * 8)) && !(rc = c->cnt.reserve((size_t)np * 4)) &&
            !(rc = c->ccnt.reserve((size_t)nc * 4)) && !(certw && (rc = c->LWE.reserve((size_t)np * 8))))
            rc = reserve_oz(c, c->H16, c->ZNZ, c->CLIVE, pipe ? nc : np);
        if (rc != LGS_ERR_NOMEM || T <= thin || n_steps <= thin) {
            if (rc) return rc;
            break;
        }
        // release the block-sized buffers (a pending look-ahead writes into a set: drop it
        // first) and retry at half the block
        if ((rc = spec_discard(c))) return rc;
        for (int si = 0; si < c->nsets; ++si) {
            auto& s = c->bset[si];
            s.Z.release();
            s.LW.release();
            s.H16.release();
            s.ZNZ.release();
            s.CLIVE.release();
        }
        c->Z.release();
        c->LW.release();
        c->cnt.release();
        c->LWE.release();
        c->H16.release();
        c->ZNZ.release();
        c->CLIVE.release();
        c->hist = decltype(c->hist){};
        maxp = std::max<int64_t>(nc * thin, maxp / 2);
        c->max_props = maxp;
        c->max_props_user = true;
    }
    // the previous call's look-ahead launch: this call's first block if it matches
    const bool no_look = c->no_look || hook_is("LGS_NO_LOOKAHEAD", 1);
    bool spec_hit = false;
    if (c->spec.valid) {
        const int64_t tb0 = std::min<int64_t>(T, n_steps);
        const auto& sp = c->spec;
        spec_hit = pipe && sp.seed == seed && sp.chain0 == first_chain && sp.step0 == first_step && sp.nc == nc &&
                   sp.Tb == tb0 && sp.ldzb == nc * tb0 + (carry ? nc : 0) && sp.zb == zb && sp.wl == wl &&
                   sp.exact == exact && sp.j == c->bset_next;
        if (!spec_hit && (rc = spec_discard(c))) return rc;
    }

    // ---- device views of the chain state (staged through device buffers for host pointers)
    void* zs = z_state;
    double* lws = logw_state;
    int32_t* init = state_init;
    int64_t* acc = accepts;
    if (!dev) {
        if ((rc = c->stage_a.reserve((size_t)nc * d * ob)) || (rc = c->stage_b.reserve((size_t)nc * 8)) ||
            (rc = c->stage_c.reserve((size_t)nc * 4)) || (rc = c->stage_d.reserve((size_t)nc * 8)))
            return rc;
        zs = c->stage_a.p;
        lws = c->stage_b.as<double>();
        init = c->stage_c.as<int32_t>();
        acc = c->stage_d.as<int64_t>();
        HIP_TRY(hipMemcpyAsync(zs, z_state, (size_t)nc * d * ob, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(lws, logw_state, nc * 8, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(init, state_init, nc * 4, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(acc, accepts, nc * 8, hipMemcpyHostToDevice, c->stream));
    }
    // per-step record: device buffers of the whole call (host pointers: copied back at the end)
    double* lwk = logw_samples;
    uint8_t* accs = accepted;
    if (!dev && (logw_samples || accepted)) {
        if ((rc = c->stage_h.reserve((size_t)std::max<int64_t>(nc * n_keep, 1) * 8)) ||
            (rc = c->stage_i.reserve((size_t)std::max<int64_t>(nc * n_steps, 1))))
            return rc;
        lwk = logw_samples ? c->stage_h.as<double>() : nullptr;
        accs = accepted ? (uint8_t*)c->stage_i.p : nullptr;
    }
    unsigned long long* mom = nullptr;
    if (moments) {
        if (dev) {
            mom = (unsigned long long*)moments;
        } else {
            if ((rc = c->stage_e.reserve((size_t)2 * d * 8))) return rc;
            mom = c->stage_e.as<unsigned long long>();
            HIP_TRY(hipMemcpyAsync(mom, moments, (size_t)2 * d * 8, hipMemcpyHostToDevice, c->stream));
        }
    }
    unsigned int* fl = c->flags.as<unsigned int>();

    // Every launch below is enqueued without a host round trip; the call waits once
    // per block (finish_or_redo).  A block whose Klein launch (or the chain states
    // carried into a 16-bit store) overflowed has its state-modifying dependants
    // skipped on the device (kAbortMask) and is redone at the wider width.
    const uint64_t next_step = first_step + (uint64_t)n_steps;  // (the look-ahead's first step)
    bool look_done = false;
    // enqueued after the call's last wait (measured: 103.6-103.9 M samples/s against
    // 101.7-102.9 M enqueued right behind the last Klein launch, whose dependants then
    // start later and hold the next launch's set longer, profiles/r05u_bench_ab.log);
    // LGS_LOOKAHEAD_EARLY=1: right behind it
    static const bool look_late = !hook_is("LGS_LOOKAHEAD_EARLY", 1);
    for (int64_t t0 = 0; t0 < n_steps || t0 == 0;) {
        bool oz_used = false;
        SetSwap sw;  // (pipe) this block's buffer set, swapped back on every exit
        if (pipe) {
            sw.c = c;
            sw.j = c->bset_next;
            sw.swap_flags();
            fl = c->flags.as<unsigned int>();
        }
        // ---- initial draws (counter step 0) of uninitialised chains (imhk.py:126-139),
        // decided on the device: the Klein launch and its application are gated by
        // "some chain has init == 0" (block 0 of the call only)
        if (t0 == 0) {
            HIP_TRY(lgs::launch::uninit_scan(init, nc, fl + kFlagWordUninit, c->stream));
            lgs::KleinArgs a = base_args(c, seed);
            a.counter_mode = 1;
            a.chain0 = (uint32_t)first_chain;
            a.step0 = 0;
            a.nt = 1;
            a.n = nc;
            a.ldz = nc;
            a.LW = c->LW.as<double>();
            if (certw) a.emax = c->EMAX.as<unsigned long long>();  // (the initial states' bound)
            a.gate = fl + kFlagWordUninit;
            bool oz0 = false;
            if ((rc = run_klein_store(c, a, exact, wl, zb, c->Z.p, true, &oz0))) return rc;
            oz_used |= oz0;
            HIP_TRY(lgs::launch::init_apply(c->Z.p, zb, init, nc, (int)d, c->LW.as<double>(), zs, ob, cm, lws,
                                            fl, c->stream));
        }
        if (n_steps == 0) {
            bool redo = false;
            if ((rc = finish_or_redo(c, oz_used, zb, redo))) return rc;
            if (redo) continue;
            break;
        }
        const int64_t Tb = std::min<int64_t>(T, n_steps - t0);
        const int64_t npb = nc * Tb;
        const int64_t first_keep = t0 / thin;  // t0 is a multiple of thin
        const int64_t kb = std::min<int64_t>(Tb / thin, n_keep - first_keep);
        if (pipe) sw.swap_store();  // the block's store, weights and history from here on
        lgs::KleinArgs a = base_args(c, seed);
        a.counter_mode = 1;
        a.chain0 = (uint32_t)first_chain;
        a.step0 = (uint32_t)(first_step + (uint64_t)t0);
        const int64_t ldzb = npb + (carry ? nc : 0);  // multiple of 4 when nc is
        a.nt = Tb;
        a.n = npb;
        a.ldz = ldzb;
        a.LW = c->LW.as<double>();
        if (certw) {
            a.LWE = c->LWE.as<double>();
            a.emax = c->EMAX.as<unsigned long long>();
        }
        bool ozb = false;
        if (pipe && spec_hit && t0 == 0) {  // the previous call's look-ahead launch is this block's
            spec_hit = false;
            c->spec.valid = false;
            for (auto& t : c->pending) t.spec = false;  // (its timers are this block's Klein launch)
            ozb = c->spec.oz;
            c->hist = c->spec.h;
            HIP_TRY(hipStreamWaitEvent(c->stream, c->spec.ev, 0));
        } else if (pipe) {  // on kstream, once the set's last reader (two blocks back) is done
            auto& bs = c->bset[sw.j];
            if (bs.free_recorded) HIP_TRY(hipStreamWaitEvent(c->kstream, bs.ev_free, 0));
            const hipStream_t cs = c->stream;
            const bool timed = c->cu_split == 0 && !c->kt_pending;  // (the CU split's measurement)
            if (timed) HIP_TRY(hipEventRecord(c->kt0, c->kstream));
            c->stream = c->kstream;
            rc = run_klein_store(c, a, exact, wl, zb, c->Z.p, true, &ozb);
            c->stream = cs;
            if (rc) return rc;
            if (timed) {
                HIP_TRY(hipEventRecord(c->kt1, c->kstream));
                c->kt_pending = true;
                c->kt_bz_ms = carry ? (double)nc * (double)kb * 8.0 * (double)d / kBzStoreBytesPerMs : 0.0;
            }
            HIP_TRY(hipEventRecord(c->ev_klein, c->kstream));
            HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_klein, 0));
        } else if ((rc = run_klein_store(c, a, exact, wl, zb, c->Z.p, true, &ozb))) {
            return rc;
        }
        // (LGS_LOOKAHEAD_EARLY) the call's last block: the next call's first block as
        // predicted, on kstream right behind this one (into the next set), before the wait
        if (pipe && !no_look && !look_late && !look_done && t0 + T >= n_steps &&
            next_step + (uint64_t)n_steps <= (1ull << 32)) {
            look_done = true;
            if ((rc = lookahead(c, (sw.j + 1) % c->nsets, seed, first_chain, next_step, nc, std::min<int64_t>(T, n_steps), carry,
                                zb, exact, wl)))
                return rc;
        }
        oz_used |= ozb;
        // chain states carried into the block's store (a state beyond 16 bits flags kFlagCarry16)
        if (carry && kb > 0)
            HIP_TRY(lgs::launch::carry_cols(zs, ob, cm, nc, (int)d, c->Z.p, zb, ldzb, npb, c->stream, fl));
        if (early) {  // every abort producer of the block is enqueued: its flag words for the host
            HIP_TRY(hipMemcpyAsync(c->fw_host, fl, 4 * lgs::kFlagWords, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipEventRecord(c->fw_ev, c->stream));
        }
        if (moments) HIP_TRY(hipMemsetAsync(c->cnt.p, 0, (size_t)npb * 4, c->stream));
        lgs::AcceptArgs aa{};
        aa.nc = nc;
        aa.T = Tb;
        aa.thin = thin;
        aa.n_keep = std::max<int64_t>(kb, 1);
        aa.seed = seed;
        aa.chain0 = (uint32_t)first_chain;
        aa.step0 = a.step0;
        aa.LW = c->LW.as<double>();
        aa.lw_state = lws;
        aa.accepts = acc;
        aa.sel = (z_samples || v_samples || zk_samples) && kb > 0 ? c->sel.as<int64_t>() : nullptr;
        aa.final_sel = c->fsel.as<int64_t>();
        aa.carry_col = carry ? npb : -1;
        aa.cnt = moments ? c->cnt.as<int32_t>() : nullptr;
        aa.cnt_carry = moments ? c->ccnt.as<int32_t>() : nullptr;
        aa.lw_keep = lwk && kb > 0 ? lwk + first_keep : nullptr;
        aa.lw_ld = n_keep;
        aa.acc_step = accs ? accs + t0 : nullptr;
        aa.acc_ld = n_steps;
        aa.abort = fl;
        aa.state_init = init;  // the step each chain's state was drawn at (certified Wang-Ling replays)
        if (certw) {  // certified Wang-Ling decisions (imhk_accept_cert_kernel)
            aa.LWE = c->LWE.as<double>();
            aa.emax = c->EMAX.as<unsigned long long>();
            aa.LWx = c->LW.as<double>();
            aa.RT = c->RT.as<double>();
            aa.Zst = c->Z.p;
            aa.zb = zb;
            aa.ldz = ldzb;
            aa.zs = zs;
            aa.ob = ob;
            aa.zs_cm = cm ? 1 : 0;
            aa.flagw = fl;
            // test hook: widened bounds force the recomputation path on many decisions
            // (clamped to >= 1: a smaller scale would shrink the bounds and void the certificate)
            const char* bs = hook("LGS_TEST_WL_BOUND_SCALE");
            aa.bscale = bs ? std::max(1.0, atof(bs)) : 1.0;
        }
        {
            Scope s(c, 2);
            HIP_TRY(lgs::launch::accept(aa, a, c->stream));
        }
        // The final-state gather rides on the moments pass unless a later step of this
        // block still reads the carried-in states (kept-state gather without carry columns).
        // (round 5) the kept states' moments from B z's digit tiles: with every step kept
        // (thin 1) the kept rows are exactly the states the moments count (proposals by
        // their keep counts, carried states through their carry columns), and B z holds
        // each row's digits in LDS anyway; the owning row tile sums each chunk's
        // coordinates over its 64 rows (bz_i8_kernel MP) and a column reduction adds
        // them up.  A carried |z| beyond two digits (B z's digit-range flag) falls back to
        // the moments pass, gated on that flag on the device.  The chains' final states
        // then come from the int16 history.  LGS_NO_BZ_MOMENTS=1: the separate pass.
        static const bool no_bz_mom = hook_is("LGS_NO_BZ_MOMENTS", 1);
        static const bool bz_f64 = hook_is("LGS_BZ_FP64", 1);
        const bool bz_mom = moments && v_samples && early && thin == 1 && kb == Tb && kb > 0 && zb == 2 &&
                            c->has_Bi8 && c->bz_mom_ok && !bz_f64 && c->hist.Z == c->Z.p && c->hist.Z &&
                            c->hist.clive != nullptr && lgs::launch::bz_moments_supported() &&
                            d % 16 == 0 && d <= lgs::kOzMaxD && npb < ((int64_t)1 << 32) && !no_bz_mom;
        const bool fuse_final = !bz_mom && moments && !((z_samples || zk_samples) && kb > 0 && !carry) &&
                                npb < ((int64_t)1 << 32);
        if (moments && !bz_mom) {
            Scope s(c, 3);
            // carried-in states first: the fused pass overwrites z_state
            HIP_TRY(lgs::launch::moments_carry(zs, ob, cm, nc, (int)d, c->ccnt.as<int32_t>(), mom, c->stream, fl));
            // the block's Klein launch wrote the int8-digit history of this store: its
            // per-block nonzero flags let the pass skip all-zero coefficient blocks
            const bool zflags = c->hist.Z == c->Z.p && c->hist.Z != nullptr;
            HIP_TRY(lgs::launch::moments_final(c->Z.p, zb, ldzb, c->cnt.as<int32_t>(), npb, Tb,
                                               fuse_final ? c->fsel.as<int64_t>() : nullptr, (int)d, mom, zs,
                                               ob, cm, nc, c->stream, fl, zflags ? c->ZNZ.as<uint8_t>() : nullptr,
                                               c->hist.lanes, (int)((16 - d % 16) % 16)));
        }
        if ((z_samples || v_samples || zk_samples) && kb > 0) {
            // kept states q = chain*kb + k, gathered coordinate-major (d x nq); chain-major
            // proposal order makes this a near-contiguous copy (outputs only: an aborted
            // attempt's values are overwritten by the redo)
            const int64_t nq = nc * kb;
            if (v_samples) {  // rows (chain, first_keep + k) of the n_chains x n_keep x d output,
                              // read straight from the proposal store through the selections
                // the fp64 replay of a digit-range overflow runs on the device, before its
                // consumers, when the host cannot replay it first: the early check, and the
                // lag sums below, which read ||v||^2 inside this call
                const bool dev_replay = early || (lag && lag->lag_v_sums && vnorm2_samples);
                const int64_t ntiles = (nq + 63) / 64, mp_ld = c->bd_cols;
                const int64_t ngw = (d + 2047) / 2048;
                unsigned int* mpl = nullptr;
                if (bz_mom) {
                    if ((rc = c->MP.reserve((size_t)ntiles * (mp_ld * 8 + ngw * 4)))) return rc;
                    mpl = (unsigned int*)(c->MP.as<unsigned long long>() + (size_t)ntiles * mp_ld);
                }
                if ((rc = run_bz(c, c->Z.p, zb, ldzb, nq, v_samples, kb, n_keep, first_keep,
                                 c->sel.as<int64_t>(), true, fl, vnorm2_samples, fn_chains * kb, dev_replay,
                                 bz_mom ? c->MP.as<unsigned long long>() : nullptr, mp_ld, mpl)))
                    return rc;
                if (bz_mom) {
                    Scope s(c, 3);
                    HIP_TRY(lgs::launch::bz_moments_reduce(c->MP.as<unsigned long long>(), mpl, ntiles, mp_ld,
                                                           (int)d, mom, fl, c->stream, fl));
                    // (the fallback, run only when B z flagged a coefficient beyond its digits)
                    HIP_TRY(lgs::launch::moments_carry(zs, ob, cm, nc, (int)d, c->ccnt.as<int32_t>(), mom,
                                                       c->stream, fl, fl));
                    HIP_TRY(lgs::launch::moments_final(c->Z.p, zb, ldzb, c->cnt.as<int32_t>(), npb, Tb, nullptr,
                                                       (int)d, mom, zs, ob, cm, nc, c->stream, fl,
                                                       c->ZNZ.as<uint8_t>(), c->hist.lanes, 0, fl));
                }
            }
            if (zk_samples)  // (the leading fn_chains chains' kept states: q < fn_chains * kb)
                HIP_TRY(lgs::launch::coord_gather(c->Z.p, zb, ldzb, c->sel.as<int64_t>(), fn_chains * kb, kb, zs, ob, cm, nc,
                                                  (int)d, (int)zk_index, zk_samples, kb, n_keep, first_keep,
                                                  c->stream, fl));
            if (lag) {  // this block's kb new values of each chain's series, in time order
                const int L = (int)lag->lag_L;
                if ((rc = c->LAGP.reserve((size_t)(L + 2) * fn_chains * 8))) return rc;
                if (lag->lag_z_sums)
                    HIP_TRY(lgs::launch::lag_update(zk_samples + first_keep, 0, n_keep, fn_chains, kb, L, 1.0,
                                                    lag->lag_z_ring, lag->lag_z_sums, c->LAGP.p, c->stream, fl));
                if (lag->lag_v_sums)
                    HIP_TRY(lgs::launch::lag_update(vnorm2_samples + first_keep, 1, n_keep, fn_chains, kb, L,
                                                    lag->lag_v_scale, lag->lag_v_ring, lag->lag_v_sums, c->LAGP.p,
                                                    c->stream, fl));
            }
            if (z_samples) {
                if ((rc = c->stage_f.reserve((size_t)nq * d * ob))) return rc;
                HIP_TRY(lgs::launch::gather_z(c->Z.p, zb, ldzb, c->sel.as<int64_t>(), nq, kb, zs, ob, cm,
                                              nc, (int)d, c->stage_f.p, 1, c->stream, fl));
                if ((rc = c->stage_g.reserve((size_t)nq * d * ob))) return rc;
                HIP_TRY(lgs::launch::transpose_out(c->stage_f.p, ob, nq, nq, (int)d, c->stage_g.p,
                                                   ob, c->stream));
                HIP_TRY(hipMemcpy2DAsync((char*)z_samples + (size_t)first_keep * d * ob,
                                         (size_t)n_keep * d * ob, c->stage_g.p, (size_t)kb * d * ob,
                                         (size_t)kb * d * ob, nc, kind_of(dev, true), c->stream));
            }
        }
        // chain states after the block (in place; carried chains keep their row)
        if (bz_mom)
            HIP_TRY(lgs::launch::final_h16(c->H16.as<int16_t>(), c->hist.lanes, c->fsel.as<int64_t>(), nc, (int)d,
                                           zs, ob, cm, c->stream, fl));
        else if (!fuse_final)
            HIP_TRY(lgs::launch::gather_z(c->Z.p, zb, ldzb, c->fsel.as<int64_t>(), nc, 1, zs, ob, cm, nc,
                                          (int)d, zs, cm, c->stream, fl));
        bool redo = false;
        if ((rc = finish_or_redo(c, oz_used, zb, redo, early))) return rc;
        if (pipe) {  // the set's readers are all enqueued (its flag words reset behind them)
            sw.release();
            fl = c->flags.as<unsigned int>();
            if (!redo) c->bset_next = (c->bset_next + 1) % c->nsets;
        }
        if (redo) continue;  // same block again (block 0: its initial draws too)
        t0 += T;
    }
    if (pipe && (rc = split_decide(c))) return rc;
    if (pipe && !no_look && look_late && next_step + (uint64_t)n_steps <= (1ull << 32))
        if ((rc = lookahead(c, c->bset_next, seed, first_chain, next_step, nc, std::min<int64_t>(T, n_steps), carry, zb,
                            exact, wl)))
            return rc;
    if (!dev) {
        HIP_TRY(hipMemcpyAsync(z_state, zs, (size_t)nc * d * ob, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(logw_state, lws, nc * 8, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(state_init, init, nc * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(accepts, acc, nc * 8, hipMemcpyDeviceToHost, c->stream));
        if (moments)
            HIP_TRY(hipMemcpyAsync(moments, mom, (size_t)2 * d * 8, hipMemcpyDeviceToHost, c->stream));
        if (logw_samples && n_keep > 0)
            HIP_TRY(hipMemcpyAsync(logw_samples, lwk, (size_t)nc * n_keep * 8, hipMemcpyDeviceToHost, c->stream));
        if (accepted && n_steps > 0)
            HIP_TRY(hipMemcpyAsync(accepted, accs, (size_t)nc * n_steps, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return LGS_OK;
}

int lgs_sample_z(lgs_ctx* c, int64_t n, const double* mu, const double* sigma, const double* u,
                 int32_t precision, int64_t* z_out, double* log_norm_out, uint32_t flags) {
    int rc = check_ctx(c, false);
    if (rc) return rc;
    if (n < 0 || !mu || !sigma || !u || !z_out) return fail(LGS_ERR_INVALID, "bad arguments");
    if (n == 0) return LGS_OK;
    for (int64_t i = 0; i < n; ++i)
        if (!(sigma[i] > 0) || !std::isfinite(sigma[i]) || !std::isfinite(mu[i]))
            return fail(LGS_ERR_INVALID, "sigma must be positive/finite and mu finite");
    DevBuf buf;
    if ((rc = buf.reserve((size_t)n * 8 * 5))) return rc;
    double* dmu = buf.as<double>();
    double* dsig = dmu + n;
    double* du = dsig + n;
    int64_t* dz = (int64_t*)(du + n);
    double* dln = (double*)(dz + n);
    HIP_TRY(hipMemcpyAsync(dmu, mu, n * 8, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(dsig, sigma, n * 8, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(du, u, n * 8, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(lgs::launch::samplez_probe(dmu, dsig, du, n, precision,
                                       (flags & LGS_BASIS_LINEAR_PROBS) ? 1 : 0,
                                       (flags & LGS_SAMPLEZ_TABLE)      ? 1
                                       : (flags & LGS_SAMPLEZ_DECISION) ? 2
                                                                        : 0,
                                       (c->libm_samplez || (flags & LGS_SAMPLEZ_LIBM)) ? nullptr
                                                                      : c->etab.as<double>(),
                                       dz, dln, c->stream));
    HIP_TRY(hipMemcpyAsync(z_out, dz, n * 8, hipMemcpyDeviceToHost, c->stream));
    if (log_norm_out)
        HIP_TRY(hipMemcpyAsync(log_norm_out, dln, n * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return LGS_OK;
}

int lgs_timing_enable(lgs_ctx* c, int enable) {
    int rc = check_ctx(c, false);
    if (rc) return rc;
    if (!c->pending.empty()) {  // timers still running belong to the old totals
        HIP_TRY(hipStreamSynchronize(c->stream));
        fold_timers(c);
    }
    c->timing = enable != 0;
    for (int k = 0; k < 7; ++k) {
        c->t_ms[k] = 0;
        c->t_n[k] = 0;
    }
    return LGS_OK;
}

int lgs_timing_get(lgs_ctx* c, int kernel, double* ms, int64_t* n) {
    if (!c) return fail(LGS_ERR_INVALID, "null context");
    if (kernel < 0 || kernel > 6) return fail(LGS_ERR_INVALID, "kernel id 0..6");
    if (!c->pending.empty()) {  // launches of an early-checked call may still be running
        int rc = check_ctx(c, false);
        if (rc) return rc;
        HIP_TRY(hipStreamSynchronize(c->stream));
        fold_timers(c);
    }
    if (ms) *ms = c->t_ms[kernel];
    if (n) *n = c->t_n[kernel];
    return LGS_OK;
}

int lgs_counter(lgs_ctx* c, int which, int reset, uint64_t* value) {
    if (!c) return fail(LGS_ERR_INVALID, "null context");
    if (which < LGS_COUNTER_RESOLVED || which > LGS_COUNTER_KLEIN_CUS)
        return fail(LGS_ERR_INVALID, "counter id 0..5");
    if (which == LGS_COUNTER_KLEIN_CUS) {
        if (value) *value = (uint64_t)c->kstream_cus;
        return LGS_OK;
    }
    uint64_t& v = which == LGS_COUNTER_RESOLVED      ? c->n_resolved
                  : which == LGS_COUNTER_FALLBACK    ? c->n_fallback
                  : which == LGS_COUNTER_ACCEPT_RESOLVED ? c->n_accept_resolved
                  : which == LGS_COUNTER_WL_MISMATCH ? c->n_wl_mismatch
                                                     : c->n_qskip;
    if (value) *value = v;
    if (reset) v = 0;
    return LGS_OK;
}

int lgs_device_info(lgs_ctx* c, char* name, int name_len, int* n_cu, int64_t* hbm) {
    int rc = check_ctx(c, false);
    if (rc) return rc;
    hipDeviceProp_t p;
    HIP_TRY(hipGetDeviceProperties(&p, c->device));
    if (name && name_len > 0) {
        snprintf(name, (size_t)name_len, "%s (%s)", p.name, p.gcnArchName);
    }
    if (n_cu) *n_cu = p.multiProcessorCount;
    if (hbm) *hbm = (int64_t)p.totalGlobalMem;
    return LGS_OK;
}

}  // extern "C"

// ============================================================ diagnostics
namespace {

int xtype_of(uint32_t flags, int& xb) {
    const uint32_t t = flags & (LGS_X_I32 | LGS_X_I64);
    if (t == (LGS_X_I32 | LGS_X_I64)) return -1;
    xb = t == LGS_X_I32 ? 4 : 8;
    return t == LGS_X_I32 ? 1 : t == LGS_X_I64 ? 2 : 0;
}

// device view of a caller buffer of `bytes` (copied in for host pointers)
int dev_in(lgs_ctx* c, bool dev, const void* p, size_t bytes, DevBuf& buf, const void*& out) {
    if (dev) {
        out = p;
        return LGS_OK;
    }
    int rc = buf.reserve(bytes);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(buf.p, p, bytes, hipMemcpyHostToDevice, c->stream));
    out = buf.p;
    return LGS_OK;
}

}  // namespace

extern "C" {

int lgs_series_stats(lgs_ctx* c, const void* x, int64_t n_series, int64_t n, int64_t group_size,
                     int64_t group_stride, int64_t series_stride, int64_t time_stride,
                     int64_t max_lag, double window_c, int64_t batch_size, double* mean_out,
                     double* c0_out, double* acf_out, double* tau_out, double* batch_means_out,
                     uint32_t flags) {
    int rc = check_ctx(c, false);
    if (rc) return rc;
    int xb = 8;
    const int xt = xtype_of(flags, xb);
    if (xt < 0) return fail(LGS_ERR_INVALID, "LGS_X_I32 and LGS_X_I64 are exclusive");
    if (n_series < 0 || n < 0 || group_size <= 0 || group_stride < 0 || series_stride < 0 ||
        time_stride < 0 || batch_size < 0)
        return fail(LGS_ERR_INVALID, "bad sizes / strides");
    if (n_series == 0) return LGS_OK;
    if (n == 0) return fail(LGS_ERR_INVALID, "empty series (the reference divides by len(x) = 0)");
    if (!x) return fail(LGS_ERR_INVALID, "null x");
    if ((acf_out || tau_out || c0_out) && max_lag < 0) return fail(LGS_ERR_INVALID, "max_lag < 0");
    if (batch_means_out && batch_size == 0) return fail(LGS_ERR_INVALID, "batch_size must be > 0");
    if (xt == 1 && n > (int64_t)1 << 32)
        return fail(LGS_ERR_INVALID, "int32 series longer than 2^32 (exact int64 sums)");
    const bool dev = flags & LGS_DEVICE_PTRS;
    const int64_t L = max_lag < n - 1 ? max_lag : n - 1;
    const int64_t nlag = L + 1, nb = batch_size ? n / batch_size : 0;
    const int64_t ng = (n_series + group_size - 1) / group_size;
    const int64_t last_s = n_series - 1;
    const size_t span = (size_t)((last_s / group_size) * group_stride + (last_s % group_size) * series_stride +
                                 (n - 1) * time_stride + 1);
    (void)ng;
    const void* X = nullptr;
    if ((rc = dev_in(c, dev, x, span * xb, c->dg_x, X))) return rc;
    // outputs: device buffers directly, or one staging block for host pointers
    const size_t o_mean = 0, o_c0 = n_series, o_tau = 2 * n_series, o_acf = 3 * n_series,
                 o_bm = o_acf + (acf_out ? (size_t)n_series * nlag : 0),
                 o_end = o_bm + (batch_means_out ? (size_t)n_series * nb : 0);
    double* O = nullptr;
    if (!dev) {
        if ((rc = c->dg_out.reserve(o_end * 8))) return rc;
        O = c->dg_out.as<double>();
    }
    lgs::SeriesArgs a{};
    a.x = X;
    a.xtype = xt;
    a.n_series = n_series;
    a.n = n;
    a.gsize = group_size;
    a.gstride = group_stride;
    a.sstride = series_stride;
    a.tstride = time_stride;
    a.max_lag = (acf_out || tau_out || c0_out) ? max_lag : -1;
    a.window_c = window_c;
    a.batch = batch_means_out ? batch_size : 0;
    a.mean = mean_out ? (dev ? mean_out : O + o_mean) : nullptr;
    a.c0 = c0_out ? (dev ? c0_out : O + o_c0) : nullptr;
    a.tau = tau_out ? (dev ? tau_out : O + o_tau) : nullptr;
    a.acf = acf_out ? (dev ? acf_out : O + o_acf) : nullptr;
    a.ld_acf = nlag;
    a.bmeans = batch_means_out ? (dev ? batch_means_out : O + o_bm) : nullptr;
    a.ld_b = nb;
    if ((rc = reset_flags(c))) return rc;
    {
        Scope s(c, 5);
        HIP_TRY(lgs::launch::series_stats(a, c->stream));
    }
    if (!dev) {
        auto back = [&](double* dst, size_t off, size_t cnt) -> int {
            if (dst) HIP_TRY(hipMemcpyAsync(dst, O + off, cnt * 8, hipMemcpyDeviceToHost, c->stream));
            return LGS_OK;
        };
        if ((rc = back(mean_out, o_mean, n_series)) || (rc = back(c0_out, o_c0, n_series)) ||
            (rc = back(tau_out, o_tau, n_series)) || (rc = back(acf_out, o_acf, (size_t)n_series * nlag)) ||
            (rc = back(batch_means_out, o_bm, (size_t)n_series * nb)))
            return rc;
    }
    return finish(c);
}

int lgs_gram(lgs_ctx* c, int64_t d, int64_t n, const void* x, int64_t ldx, const void* shift,
             void* sum_out, void* gram_out, uint32_t flags) {
    int rc = check_ctx(c, false);
    if (rc) return rc;
    int xb = 8;
    const int xt = xtype_of(flags, xb);
    if (xt < 0 || d <= 0 || n < 0 || d > (1 << 20)) return fail(LGS_ERR_INVALID, "bad d / n / type");
    if (!gram_out && !sum_out) return LGS_OK;
    if (n == 0) return LGS_OK;
    if (!x) return fail(LGS_ERR_INVALID, "null x");
    const bool dev = flags & LGS_DEVICE_PTRS, cm = flags & LGS_COORD_MAJOR;
    if (cm ? ldx < n : ldx != d) return fail(LGS_ERR_INVALID, "ldx: >= n (coordinate-major) or == d (row-major)");
    if ((rc = reset_flags(c))) return rc;
    const size_t xbytes = cm ? ((size_t)(d - 1) * ldx + n) * xb : (size_t)n * d * xb;
    const void* Xin = nullptr;
    if ((rc = dev_in(c, dev, x, xbytes, c->dg_x, Xin))) return rc;
    const void* SH = nullptr;
    if (shift && (rc = dev_in(c, dev, shift, (size_t)d * 8, c->dg_c, SH))) return rc;
    // accumulators: the caller's (device) or staged copies of the host values (ADDED to)
    void* G = gram_out;
    void* S = sum_out;
    const size_t gbytes = (size_t)d * d * 8, sbytes = (size_t)d * 8;
    if (!dev || !gram_out || !sum_out) {
        if ((rc = c->dg_a.reserve(gbytes)) || (rc = c->dg_b.reserve(sbytes))) return rc;
        if (!dev || !gram_out) {
            G = c->dg_a.p;
            if (gram_out)
                HIP_TRY(hipMemcpyAsync(G, gram_out, gbytes, hipMemcpyHostToDevice, c->stream));
            else
                HIP_TRY(hipMemsetAsync(G, 0, gbytes, c->stream));
        }
        if (!dev || !sum_out) {
            S = c->dg_b.p;
            if (sum_out)
                HIP_TRY(hipMemcpyAsync(S, sum_out, sbytes, hipMemcpyHostToDevice, c->stream));
            else
                HIP_TRY(hipMemsetAsync(S, 0, sbytes, c->stream));
        }
    }
    bool valu = xt == 0;
    if (!valu) {  // int8 digit planes, then the MFMA Gram (exact while |x - shift| <= 32639)
        const int64_t ldp = (n + 63) / 64 * 64, dpad = (d + 127) / 128 * 128;
        if ((rc = c->dg_y.reserve((size_t)2 * dpad * ldp))) return rc;
        int8_t* Ph = c->dg_y.as<int8_t>();
        int8_t* Pl = Ph + (size_t)dpad * ldp;
        unsigned int f = 0;
        {
            // the planes pass is gated on the packing's range flag on the device, so both
            // are enqueued before the one synchronisation
            Scope s(c, 4);
            HIP_TRY(lgs::launch::gram_pack(Xin, xt, cm, ldx, (int)d, n, (const long long*)SH, Ph, Pl, ldp,
                                           c->flags.as<unsigned int>(), c->stream));
            HIP_TRY(lgs::launch::gram_planes(Ph, Pl, ldp, (int)d, G, S, c->stream, c->flags.as<unsigned int>()));
            if (dev && gram_out && sum_out && cm && c->stream != c->own) {
                // caller-owned device accumulators, coordinate-major input, on a stream the
                // caller set (lgs_set_stream: it orders its own work after ours): the exact
                // VALU replay is gated on the same flag, so nothing needs the host -- no
                // synchronisation (the next call's flag reset is stream-ordered)
                HIP_TRY(lgs::launch::gram(Xin, xt, ldx, (int)d, n, SH, G, S, c->stream,
                                          c->flags.as<unsigned int>()));
                return LGS_OK;
            }
        }
        HIP_TRY(hipMemcpyAsync(&f, c->flags.p, sizeof(f), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (f & lgs::kFlagI8Range) {
            valu = true;  // some |x - shift| > 32639: exact int64 VALU (the planes pass returned at once)
            HIP_TRY(hipMemsetAsync(c->flags.p, 0, 16, c->stream));
        }
    }
    if (valu) {
        const void* Xc = Xin;
        int64_t ld = ldx;
        if (!cm) {  // row-major -> coordinate-major (8-byte elements move as bit patterns)
            if ((rc = c->dg_t.reserve((size_t)n * d * xb))) return rc;
            HIP_TRY(lgs::launch::to_coord_major(Xin, xb, n, (int)d, c->dg_t.p, xb, n, c->stream));
            Xc = c->dg_t.p;
            ld = n;
        }
        Scope s(c, 4);
        HIP_TRY(lgs::launch::gram(Xc, xt, ld, (int)d, n, SH, G, S, c->stream));
    }
    if (!dev) {
        if (gram_out) HIP_TRY(hipMemcpyAsync(gram_out, G, gbytes, hipMemcpyDeviceToHost, c->stream));
        if (sum_out) HIP_TRY(hipMemcpyAsync(sum_out, S, sbytes, hipMemcpyDeviceToHost, c->stream));
    }
    return finish(c);
}

int lgs_jump_distance(lgs_ctx* c, int64_t n, int64_t d, const void* x, int64_t ld, double* out,
                      uint32_t flags) {
    int rc = check_ctx(c, false);
    if (rc) return rc;
    int xb = 8;
    const int xt = xtype_of(flags, xb);
    if (xt < 0 || n < 0 || d <= 0 || ld < d) return fail(LGS_ERR_INVALID, "bad arguments");
    if (n < 2) return LGS_OK;
    if (!x || !out) return fail(LGS_ERR_INVALID, "null buffer");
    const bool dev = flags & LGS_DEVICE_PTRS;
    if ((rc = reset_flags(c))) return rc;
    const void* X = nullptr;
    if ((rc = dev_in(c, dev, x, ((size_t)(n - 1) * ld + d) * xb, c->dg_x, X))) return rc;
    double* O = out;
    if (!dev) {
        if ((rc = c->dg_out.reserve((size_t)(n - 1) * 8))) return rc;
        O = c->dg_out.as<double>();
    }
    HIP_TRY(lgs::launch::jump(X, xt, n, (int)d, ld, O, c->stream));
    if (!dev) HIP_TRY(hipMemcpyAsync(out, O, (size_t)(n - 1) * 8, hipMemcpyDeviceToHost, c->stream));
    return finish(c);
}

int lgs_marginal_tvd(lgs_ctx* c, int64_t d, const void* x1, int64_t n1, const void* x2, int64_t n2,
                     double* tvd_out, uint32_t flags) {
    int rc = check_ctx(c, false);
    if (rc) return rc;
    int xb = 8;
    const int xt = xtype_of(flags, xb);
    if (xt < 0 || d <= 0 || n1 <= 0 || n2 <= 0) return fail(LGS_ERR_INVALID, "bad arguments");
    if (!x1 || !x2 || !tvd_out) return fail(LGS_ERR_INVALID, "null buffer");
    const bool dev = flags & LGS_DEVICE_PTRS;
    if ((rc = reset_flags(c))) return rc;
    const void *X1 = nullptr, *X2 = nullptr;
    if ((rc = dev_in(c, dev, x1, (size_t)n1 * d * xb, c->dg_x, X1)) ||
        (rc = dev_in(c, dev, x2, (size_t)n2 * d * xb, c->dg_y, X2)))
        return rc;
    // per-coordinate value range over both sets
    if ((rc = c->dg_a.reserve((size_t)(3 * d + 1) * 8))) return rc;
    long long* mn = c->dg_a.as<long long>();
    long long* mx = mn + d;
    long long* off = mx + d;
    std::vector<long long> h_mn(d, LLONG_MAX), h_mx(d, LLONG_MIN), h_off(d + 1, 0);
    HIP_TRY(hipMemcpyAsync(mn, h_mn.data(), d * 8, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(mx, h_mx.data(), d * 8, hipMemcpyHostToDevice, c->stream));
    unsigned int* fl = c->flags.as<unsigned int>();
    HIP_TRY(lgs::launch::tvd_minmax(X1, xt, n1, (int)d, mn, mx, fl, c->stream));
    HIP_TRY(lgs::launch::tvd_minmax(X2, xt, n2, (int)d, mn, mx, fl, c->stream));
    unsigned int f = 0;
    HIP_TRY(hipMemcpyAsync(h_mn.data(), mn, d * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(h_mx.data(), mx, d * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(&f, fl, sizeof(f), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (f & lgs::kFlagNonFinite)
        return fail(LGS_ERR_INVALID, "marginal TVD: samples must be integer-valued (discrete case)");
    const long long kMaxBins = 1LL << 28;
    for (int64_t i = 0; i < d; ++i) {
        const long long w = h_mx[i] - h_mn[i] + 1;
        if (w <= 0 || w > kMaxBins || h_off[i] + w > kMaxBins)
            return fail(LGS_ERR_INVALID, "marginal TVD: value ranges exceed 2^28 bins in total");
        h_off[i + 1] = h_off[i] + w;
    }
    const long long bins = h_off[d];
    HIP_TRY(hipMemcpyAsync(off, h_off.data(), (d + 1) * 8, hipMemcpyHostToDevice, c->stream));
    if ((rc = c->dg_b.reserve((size_t)bins * 8))) return rc;
    unsigned int* c1 = c->dg_b.as<unsigned int>();
    unsigned int* c2 = c1 + bins;
    HIP_TRY(hipMemsetAsync(c1, 0, (size_t)bins * 8, c->stream));
    HIP_TRY(lgs::launch::tvd_hist(X1, xt, n1, (int)d, mn, off, c1, c->stream));
    HIP_TRY(lgs::launch::tvd_hist(X2, xt, n2, (int)d, mn, off, c2, c->stream));
    double* O = tvd_out;
    if (!dev) {
        if ((rc = c->dg_out.reserve((size_t)d * 8))) return rc;
        O = c->dg_out.as<double>();
    }
    HIP_TRY(lgs::launch::tvd_sum(c1, c2, off, (int)d, n1, n2, O, c->stream));
    if (!dev) HIP_TRY(hipMemcpyAsync(tvd_out, O, (size_t)d * 8, hipMemcpyDeviceToHost, c->stream));
    return finish(c);
}

int lgs_column_range(lgs_ctx* c, int64_t d, const void* x, int64_t n, double* min_out, double* max_out,
                     uint32_t flags) {
    int rc = check_ctx(c, false);
    if (rc) return rc;
    int xb = 8;
    const int xt = xtype_of(flags, xb);
    if (xt < 0 || d <= 0 || n <= 0) return fail(LGS_ERR_INVALID, "bad arguments");
    if (!x || !min_out || !max_out) return fail(LGS_ERR_INVALID, "null buffer");
    const bool dev = flags & LGS_DEVICE_PTRS;
    if ((rc = reset_flags(c))) return rc;
    const void* X = nullptr;
    if ((rc = dev_in(c, dev, x, (size_t)n * d * xb, c->dg_x, X))) return rc;
    if ((rc = c->dg_a.reserve((size_t)4 * d * 8))) return rc;
    long long* mn = c->dg_a.as<long long>();
    long long* mx = mn + d;
    std::vector<long long> init(2 * d);
    for (int64_t i = 0; i < d; ++i) {
        init[i] = LLONG_MAX;
        init[d + i] = LLONG_MIN;
    }
    HIP_TRY(hipMemcpyAsync(mn, init.data(), (size_t)2 * d * 8, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(lgs::launch::hist_range(X, xt, n, (int)d, mn, mx, c->flags.as<unsigned int>(), c->stream));
    double* lo = dev ? min_out : (double*)(mx + d);
    double* hi = dev ? max_out : lo + d;
    HIP_TRY(lgs::launch::hist_keys_to_f64(mn, mx, (int)d, lo, hi, c->stream));
    if (!dev) {
        HIP_TRY(hipMemcpyAsync(min_out, lo, (size_t)d * 8, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(max_out, hi, (size_t)d * 8, hipMemcpyDeviceToHost, c->stream));
    }
    rc = finish(c);
    if (rc == LGS_ERR_NONFINITE)
        return fail(LGS_ERR_NONFINITE, "column range: non-finite value (or |integer| > 2^53)");
    return rc;
}

int lgs_histogram(lgs_ctx* c, int64_t d, const void* x, int64_t n, int64_t bins, const double* edges,
                  const double* first_denom, int64_t* counts_out, uint32_t flags) {
    int rc = check_ctx(c, false);
    if (rc) return rc;
    int xb = 8;
    const int xt = xtype_of(flags, xb);
    if (xt < 0 || d <= 0 || n < 0 || bins <= 0 || d * bins > (1LL << 31))
        return fail(LGS_ERR_INVALID, "bad arguments");
    if ((n > 0 && !x) || !edges || !first_denom || !counts_out) return fail(LGS_ERR_INVALID, "null buffer");
    const bool dev = flags & LGS_DEVICE_PTRS;
    if ((rc = reset_flags(c))) return rc;
    const void *X = nullptr, *E = nullptr, *FD = nullptr;
    if ((rc = dev_in(c, dev, x, (size_t)n * d * xb, c->dg_x, X)) ||
        (rc = dev_in(c, dev, edges, (size_t)d * (bins + 1) * 8, c->dg_y, E)) ||
        (rc = dev_in(c, dev, first_denom, (size_t)d * 2 * 8, c->dg_a, FD)))
        return rc;
    unsigned long long* cnt = (unsigned long long*)counts_out;
    if (!dev) {
        if ((rc = c->dg_b.reserve((size_t)d * bins * 8))) return rc;
        cnt = c->dg_b.as<unsigned long long>();
    }
    HIP_TRY(hipMemsetAsync(cnt, 0, (size_t)d * bins * 8, c->stream));
    HIP_TRY(lgs::launch::hist_counts(X, xt, n, (int)d, bins, (const double*)E, (const double*)FD, cnt, c->stream));
    if (!dev) HIP_TRY(hipMemcpyAsync(counts_out, cnt, (size_t)d * bins * 8, hipMemcpyDeviceToHost, c->stream));
    return finish(c);
}

}  // extern "C"

// ============================================================ decoding
namespace {

// Shared driver of lgs_nearest_plane / lgs_round_decode: per chunk of targets,
// W = M t on fp64 MFMA (M = Q^T or B^{-1}), then the nearest-plane walk or the
// rounding, then z / v outputs as lgs_klein writes them.
int run_decode(lgs_ctx* c, bool plane, int64_t n, const double* targets, void* z_out, double* v_out,
               uint32_t flags) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (n < 0) return fail(LGS_ERR_INVALID, "n < 0");
    if (n == 0) return LGS_OK;
    if (!targets) return fail(LGS_ERR_INVALID, "null targets");
    if (plane ? !c->has_q : !c->has_binv)
        return fail(LGS_ERR_STATE, plane ? "nearest plane needs Q (lgs_set_decoder)"
                                         : "rounding decode needs B^-1 (lgs_set_decoder)");
    if (v_out && !c->has_B) return fail(LGS_ERR_STATE, "v_out requires B");
    const bool dev = flags & LGS_DEVICE_PTRS, z64 = flags & LGS_Z64, cm = flags & LGS_COORD_MAJOR;
    const int64_t d = c->d;
    const int ob = z64 ? 8 : 4;
    if ((rc = reset_flags(c))) return rc;
    const int64_t chunk = std::min<int64_t>(n, std::max<int64_t>(256, ((int64_t)1 << 27) / d));
    if ((rc = c->dg_x.reserve((size_t)chunk * d * 8)) || (rc = c->dg_y.reserve((size_t)chunk * d * 8)) ||
        (rc = c->Z.reserve((size_t)chunk * d * ob)))
        return rc;
    if (!dev) {
        if ((rc = c->stage_a.reserve((size_t)chunk * d * std::max(ob, 8)))) return rc;
        if (v_out && (rc = c->V.reserve((size_t)chunk * d * 8))) return rc;
    }
    double* X = c->dg_x.as<double>();   // targets, coordinate-major (d x m)
    double* Y = c->dg_y.as<double>();   // M t, row-major (m x d), then coordinate-major in X
    for (int64_t off = 0; off < n; off += chunk) {
        const int64_t m = std::min<int64_t>(chunk, n - off);
        // targets -> X (d x m)
        if (cm) {
            for (int64_t i = 0; i < d; ++i)
                HIP_TRY(hipMemcpyAsync(X + (size_t)i * m, targets + (size_t)i * n + off, (size_t)m * 8,
                                       kind_of(true, dev), c->stream));
        } else {
            const double* src = targets + (size_t)off * d;
            if (!dev) {
                HIP_TRY(hipMemcpyAsync(c->stage_a.p, src, (size_t)m * d * 8, hipMemcpyHostToDevice, c->stream));
                src = c->stage_a.as<double>();
            }
            HIP_TRY(lgs::launch::to_coord_major(src, 8, m, (int)d, X, 8, m, c->stream));
        }
        HIP_TRY(lgs::launch::gemm_f64(X, m, plane ? c->DQ.as<double>() : c->DBIT.as<double>(), (int)d, m, Y,
                                      c->stream));
        HIP_TRY(lgs::launch::to_coord_major(Y, 8, m, (int)d, X, 8, m, c->stream));
        void* Zp = c->Z.p;
        if (plane) {
            const double* co = c->coord.as<double>();
            HIP_TRY(lgs::launch::nearest_plane((int)d, m, c->panel, c->RP.as<double>(), c->RC.as<double>(),
                                               co + d, X, m, ob, Zp, m, c->flags.as<unsigned int>(),
                                               c->stream));
        } else {
            HIP_TRY(lgs::launch::round_coeffs(X, m, (int)d, m, ob, Zp, m, c->flags.as<unsigned int>(),
                                              c->stream));
        }
        if (z_out) {
            if (cm) {
                for (int64_t i = 0; i < d; ++i)
                    HIP_TRY(hipMemcpyAsync((char*)z_out + ((size_t)i * n + off) * ob, (char*)Zp + (size_t)i * m * ob,
                                           (size_t)m * ob, kind_of(dev, true), c->stream));
            } else {
                void* dst = dev ? (char*)z_out + (size_t)off * d * ob : c->stage_a.p;
                HIP_TRY(lgs::launch::transpose_out(Zp, ob, m, m, (int)d, dst, ob, c->stream));
                if (!dev)
                    HIP_TRY(hipMemcpyAsync((char*)z_out + (size_t)off * d * ob, dst, (size_t)m * d * ob,
                                           hipMemcpyDeviceToHost, c->stream));
            }
        }
        if (v_out) {
            double* V = dev ? v_out + (size_t)off * d : c->V.as<double>();
            if ((rc = run_bz(c, Zp, ob, m, m, V))) return rc;
            if ((rc = settle_bz(c))) return rc;
            if (!dev)
                HIP_TRY(hipMemcpyAsync(v_out + (size_t)off * d, V, (size_t)m * d * 8, hipMemcpyDeviceToHost,
                                       c->stream));
        }
        if ((rc = finish(c))) return rc;
    }
    return finish(c);
}

}  // namespace

extern "C" {

int lgs_set_decoder(lgs_ctx* c, const double* Q, const double* Binv) {
    int rc = check_ctx(c);
    if (rc) return rc;
    const int64_t d = c->d;
    const size_t bytes = (size_t)d * d * 8;
    HIP_TRY(hipStreamSynchronize(c->stream));  // (as lgs_set_basis: in-flight work may read the buffers)
    if (c->kstream) HIP_TRY(hipStreamSynchronize(c->kstream));
    if (Q) {
        if ((rc = c->DQ.reserve(bytes))) return rc;
        HIP_TRY(hipMemcpy(c->DQ.p, Q, bytes, hipMemcpyHostToDevice));  // gemm_f64 reads Q[c][r]
        c->has_q = true;
    }
    if (Binv) {
        std::vector<double> t((size_t)d * d);
        for (int64_t r = 0; r < d; ++r)
            for (int64_t k = 0; k < d; ++k) t[(size_t)k * d + r] = Binv[(size_t)r * d + k];
        if ((rc = c->DBIT.reserve(bytes))) return rc;
        HIP_TRY(hipMemcpy(c->DBIT.p, t.data(), bytes, hipMemcpyHostToDevice));
        c->has_binv = true;
    }
    return LGS_OK;
}

int lgs_nearest_plane(lgs_ctx* c, int64_t n, const double* targets, void* z_out, double* v_out,
                      uint32_t flags) {
    return run_decode(c, true, n, targets, z_out, v_out, flags);
}

int lgs_round_decode(lgs_ctx* c, int64_t n, const double* targets, void* z_out, double* v_out,
                     uint32_t flags) {
    return run_decode(c, false, n, targets, z_out, v_out, flags);
}

}  // extern "C"
