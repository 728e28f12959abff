// lgs_kernels.h -- internal interface between the C-ABI (lgs_capi.hip) and the
// kernels (lgs_kernels.hip).  Not part of the public ABI (see include/lgs.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Round-6 defaults of the Klein kernel's near field, measured together under the
// scheduler flags (Makefile) with identical outputs: the record laid out decision-first
// with its near-field coefficients read last (LGS_REC_L2), the record's LDS reads left
// to the scheduler instead of pinned per register (LGS_REC_NOPIN), and the Philox round
// keys left to loop-invariant motion (LGS_PHILOX_HOIST).  Each alone is within noise;
// together the bench 117.0-117.4 -> 118.9-119.6 M samples/s and Klein 28.84-28.93 ->
// 28.20-28.34 ms per 2^22 block (profiles/r06au_bench_variants.log), C3 / C4 / C5 Klein
// -1.6 / -1.0 / -1.3 % at 2^20 samples and C1 / C2 +1.7 / +1.2 % (r06av_call_kbench.log).
// LGS_R6_OFF restores the round-5 forms.
#ifndef LGS_R6_OFF
#ifndef LGS_REC_L2
#define LGS_REC_L2 1
#endif
#ifndef LGS_REC_NOPIN
#define LGS_REC_NOPIN 1
#endif
#ifndef LGS_PHILOX_HOIST
#define LGS_PHILOX_HOIST 1
#endif
#endif

namespace lgs {

constexpr unsigned int kFlagNonFinite = 1u;  // a conditional mean was NaN/inf
constexpr unsigned int kFlagOverflow = 2u;   // |z| >= 2^31 with an int32 store
constexpr unsigned int kFlagI8Range = 4u;    // |z| > 32639: int8-digit B z must be redone in fp64
constexpr unsigned int kFlagOverflow16 = 8u; // |z| > 32767 in a 16-bit internal store
constexpr unsigned int kFlagCarry16 = 16u;   // a chain state carried into a 16-bit store does not fit
// lgs_imhk enqueues a block's Klein launch and its dependants without waiting: the
// dependants that modify caller state (acceptance, moments, state gathers, initial
// draws) return immediately when the launch set one of these, and the block is
// redone at the wider width after the call's single synchronisation
constexpr unsigned int kAbortMask = kFlagOverflow16 | kFlagCarry16;
// flags[1] of a launch: coordinates whose decision at the blocked-order mean could
// not be certified and was redone at the reference-order mean (lgs_device.h)
constexpr int kFlagWordResolved = 1;
constexpr int kFlagWordUninit = 4;      // lgs_imhk: some chain needs its initial draw
constexpr int kFlagWordCheckpoint = 5;  // lgs_imhk: resolved count before the block's Klein launch

constexpr int kErfTabLast = 512;
constexpr int kCoefStride = 18;  // doubles per grid point of the coefficient table (lgs_device.h CoefTab)  // SampleZ erf/exp table: y_j = j/64, j = 0..kErfTabLast (y <= 8)

// Per-coordinate SampleZ constants (kSzcStride doubles per coordinate, built by
// the host in lgs_set_basis; lgs_device.h sample_z_coord):
//   [0] sigma_i  [1] 1/sigma_i  [2] kind  [3] sc = sigma*sqrt(pi/2)  [4] 1/sc
//   [5] sigma*sqrt(2)  [6] rf*sigma (window half-width, klein.py:113-120)
//   [7] S, [8] base (kind kSzClosed); [7] of the capped kind: 1 when sigma >= 360
//   (series erf / exp over the whole window, lgs_device.h PolyErf)
//   [kSzS..kSzS+kSzDeg] / [kSzB..kSzB+kSzDeg]: monomial coefficients in
//   m = mu - rint(mu) of S(m) / base(m) (kind kSzCapped)
//   [kSzCa], [kSzCb]: decision certificate of the blocked kernels (lgs_device.h
//   certified decisions): |mu_fast - mu_ref| <= Ca + Cb * sum_{j>i} |z_j| + 6e-16 |mu|
//   [7] of the small kind: 1 when points entering / leaving the window at its ends
//   can carry more than 2^-60 of the mass (the certificate then checks the ends)
constexpr int kSzDeg = 5;  // degree 4 already reaches the fp64 floor for sigma in [50, 1e6]
constexpr int kSzS = 9;
constexpr int kSzB = kSzS + kSzDeg + 1;
constexpr int kSzCa = kSzB + kSzDeg + 1;  // 21
constexpr int kSzCb = kSzCa + 1;
constexpr int kSzUsed = kSzCb + 1;  // 23
constexpr int kSzcStride = 24;
// Klein-path record per coordinate (kRecStride doubles): the SampleZ constants
// [0, kSzUsed), then c', 1/R_ii, R_ii/sigma, 1/sigma_i^ref, lterm, and the 15
// near-field coefficients R[i-1-m][i] of the coordinate's 16-row sub-panel.
// Staged into LDS once per 32-row panel by klein_mfma_kernel.
#ifdef LGS_REC_L2
// (variant) the dispatch code and the weight constants before the near-field
// coefficients: the step's decision then waits for the first 15 of the record's 22
// 16-byte reads, and Rs[1..14] arrive while it runs
constexpr int kRecCp = kSzUsed, kRecIrii = kSzUsed + 1, kRecDisp = kSzUsed + 2, kRecRos = kSzUsed + 3,
              kRecIsr = kSzUsed + 4, kRecLterm = kSzUsed + 5, kRecCbC = kSzUsed + 6, kRecRs = kSzUsed + 7;
constexpr int kRecScale = kRecRs + 15;
constexpr int kRecSpec = kRecScale + 1;
#else
constexpr int kRecCp = kSzUsed, kRecIrii = kSzUsed + 1, kRecRos = kSzUsed + 2,
              kRecIsr = kSzUsed + 3, kRecLterm = kSzUsed + 4, kRecRs = kSzUsed + 5;
// SampleZ dispatch code of the coordinate (host): 0.0 = small kind with one dominant
// window point possible (q[7] == 0), 1.0 = capped kind with sigma >= 360 (q[7] == 1),
// 2.0 = anything else (sigma_i == 0 included); inside the hot record batch
constexpr int kRecDisp = kRecRs + 15;
// int8-digit far field (klein_mfma_kernel OZ): row scale 2^E_i of the
// coordinate's row over its panel's far columns
constexpr int kRecScale = kRecRs + 16;
#endif
// 1.0 when the coordinate's 16-row sub-panel is whole and all its coordinates are
// of the small kind with one dominant window point possible (q[7] == 0): the
// sub-panel is then decided speculatively in parallel (klein_mfma_kernel)
#ifndef LGS_REC_L2
constexpr int kRecSpec = kRecScale + 1;
// Cb of the certificate for a mean whose far field used only the 3 most significant
// R digits (reference mode, panels of two speculative sub-panels: klein_mfma_kernel)
constexpr int kRecCbC = kRecScale + 2;
#endif
constexpr int kRecStride = 48;  // 384 bytes, 16-byte multiple
#ifndef LGS_BZ_BN
#define LGS_BZ_BN 128
#endif
// B z (bz_i8_kernel): coordinates per workgroup tile (128, or 64: half the
// accumulators per wave, twice the workgroups)
constexpr int kBzBN = LGS_BZ_BN;
static_assert(kRecCbC < kRecStride, "record layout");
constexpr int kOzCoarse = 4;  // R digits of the far field in coarse panels
// int8-digit far field layout: per 32-row panel pk >= 1 (K = 32 pk far columns,
// ceil(K/64) chunks of 64): [chunk][row tile t][digit a][lane][16 bytes]
#ifndef LGS_OZ_DIGITS
#define LGS_OZ_DIGITS 6
#endif
constexpr int kOzDigits = LGS_OZ_DIGITS;  // R digits: 48 significant bits (the rounding adds 128 u M to Cb, lgs_set_basis)
constexpr int kOzMaxD = 32768;  // int32 class sums stay exact: 2 * K * 2^14 < 2^31
constexpr int kSzRound = 0;    // sigma_i < 1e-10: round(mu), no draw
constexpr int kSzSmall = 1;    // sigma_i < 4: <= 4-point exponent path / table walk
constexpr int kSzClosed = 2;   // uncapped window of +-rf*sigma, rf >= 9: S = 2 sc, base = -sc
constexpr int kSzCapped = 3;   // window capped to rint(mu) +- 500: S(m), base(m) polynomials
constexpr int kSzGeneric = 4;  // anything else: both window ends evaluated per draw

constexpr int kKernelExact = 0;  // reference-order back-substitution
constexpr int kKernelValu = 1;   // blocked panel kernel, VALU far field
constexpr int kKernelMfma = 2;   // blocked panel kernel, fp64 MFMA far field

// Per-launch arguments of the Klein samplers.  Per-coordinate arrays (length d):
//   cp      c' = Q^T c
//   rii     R_ii (> 0 after the sign fix of klein.py:69-73)
//   sig     effective SampleZ sigma: sigma/R_ii, clamped to 1e6 above 1e10,
//           0 when sigma/R_ii < 1e-10 (deterministic rounding)
//   sig_ref sigma/R_ii unclamped (reference-mode weight, klein.py:255-263)
//   lterm   0.5*log(2*pi) + log(sig_ref)
//   irii    1/R_ii, ros = R_ii/sigma, isr = 1/sig_ref (reciprocal forms for the
//           fast kernels; the exact-order kernel divides like the reference)
struct KleinArgs {
    int d;
    int precision;
    int linear_probs;
    int counter_mode;  // 0: lane p -> sample base+p; 1: chain0 + p/nt, step0 + p%nt (chain-major)
    const double* cp;
    const double* rii;
    const double* sig;
    const double* sig_ref;
    const double* lterm;
    const double* irii;
    const double* ros;
    const double* isr;
    const double* R;     // row-major R (reference-order means of uncertified decisions)
    double sigma;
    double z1cap;        // 32-row panels: certificate bound on sum_j |z_j| (verified per sub-panel)
    unsigned long long* z1max;  // 32-row panels: atomicMax of the samples' sum |z_j| (fp64 bits)
    uint64_t seed;
    uint64_t base;
    uint32_t chain0;
    uint32_t step0;
    int64_t nt;
    int64_t n;
    int64_t ldz;
    double* LW;
    unsigned int* flags;
    const double* etab;  // SampleZ erf/exp table (nullptr: ocml libm path)
    const double* etab2; // its Taylor-coefficient form (lgs_device.h CoefTab)
    const double* szc;   // per-coordinate SampleZ constants (nullptr: generic sample_z)
    const double* cert;  // per coordinate {Ca, Cb} of the decision certificate (kSzCa / kSzCb)
    const double* crec;  // per-coordinate records (kRecStride doubles, layout above)
    // int8-digit far field (nullptr rd: fp64 MFMA far field)
    const int8_t* rd;        // R digit fragments, all panels
    const int64_t* rd_off;   // byte offset of panel pk in rd
    int16_t* h16;            // coefficient history, [(i + h16_shift)/16][lane][16] int16
    int h16_shift;           // (16 - d % 16) % 16
    int64_t h16_lanes;       // lanes per 16-coordinate block (>= n)
    uint8_t* znz;            // nullable (with h16): [(i + h16_shift)/16][lane] 1 when the lane's z of
                             // that block has a nonzero (B z skips chunks that are all zero)
    const double* rx;    // per 32-row panel: 16x16 block R[p_hi-32.., p_hi-16..] as MFMA A fragments
    const unsigned int* gate;  // nullable: when *gate == 0 every block returns at once (initial draws
                               // of lgs_imhk when no chain needs one, decided on the device)
    // Wang-Ling mode, blocked kernels (nullable): per sample a bound E >= |LW - LW_ref|,
    // LW_ref = the log weight at the reference-order means (what klein_exact_kernel
    // returns), from the certificate's bound on each mean (lgs_kernels.hip wl_bound_*)
    double* LWE;
    unsigned long long* emax;  // nullable: atomicMax of those bounds (fp64 bits, E >= 0)
    // q-panel skip (reference mode, int8-digit far field; nullable): per 32-row panel the
    // largest ||z_W||^2 for which every row's mean is certified to give z = 0 without
    // computing it (lgs_set_basis), < 0 where it does not apply
    const double* qz2;
    // nullable (with h16, d % 16 == 0): per wave of the launch, bit c & 31 of word
    // clive[(c >> 5) * clive_ld + wave] set when some lane has a nonzero z in the
    // 64-coordinate chunk c (zeroed before the launch; B z's chunk skipping)
    unsigned int* clive;
    int64_t clive_ld;
};

// Counter / check words of the context's flag buffer used by the certified
// Wang-Ling accept decisions (imhk_accept_kernel)
constexpr int kFlagWordAcceptResolved = 6;  // decisions redone at reference-order weights
constexpr int kFlagWordWLMismatch = 7;      // recomputed draws that did not reproduce the stored z (a bug)
constexpr int kFlagWordQSkip = 8;           // (wave, panel) pairs of the q-panel skip (klein_mfma_kernel)
constexpr int kFlagWords = 16;              // the flag buffer: 64 bytes

struct AcceptArgs {
    int64_t nc;
    int64_t T;
    int64_t thin;
    int64_t n_keep;
    uint64_t seed;
    uint32_t chain0;
    uint32_t step0;
    const double* LW;
    double* lw_state;
    int64_t* accepts;
    int64_t* sel;        // nullable, nc x n_keep
    int64_t* final_sel;  // nc
    int32_t* cnt;        // nullable, per proposal (zeroed by caller)
    int32_t* cnt_carry;  // nullable, per chain
    int64_t carry_col;   // >= 0: sel of a state carried in from before the block = carry_col + chain
    double* lw_keep;     // nullable: log weight of kept state k of chain c at lw_keep[c * lw_ld + k]
    int64_t lw_ld;
    uint8_t* acc_step;   // nullable: 1 where step t of chain c accepted, at acc_step[c * acc_ld + t]
    int64_t acc_ld;
    const unsigned int* abort;  // nullable: return at once when *abort & kAbortMask
    // Certified Wang-Ling decisions (LWE non-null, blocked kernels): each decision is
    // taken only when it is the same for every pair of weights within the bounds
    // LWE (proposals) / *emax (chain states carried into the block) of the stored
    // ones; otherwise both weights are recomputed in the reference's order by the
    // wave (wl_exact_wave) and written back with bound 0.
    double* LWE;
    const unsigned long long* emax;
    double* LWx;            // = LW, writable (recomputed weights)
    const double* RT;       // R transposed, d x d (RT[j * d + i] = R[i][j])
    const void* Zst;        // proposal store (coordinate-major, column p, ld ldz, zb-byte elements)
    int zb;
    int64_t ldz;
    const void* zs;         // chain states carried into the block (caller's layout)
    int ob;
    int zs_cm;
    unsigned int* flagw;    // the context's flag words (kFlagWordAcceptResolved, kFlagWordWLMismatch)
    double bscale;          // bounds x bscale (1; a test hook widens them to force recomputations)
    // nullable: the chains' state_init words (lgs.h): >= kInitStep0 = the state is the
    // chain's draw at counter step (word - kInitStep0), so a carried-in state's weight is
    // recomputed with its own uniforms; 1 = initialised, step unknown.  Updated for the
    // chains whose state changes in the block.
    int32_t* state_init;
};
constexpr int32_t kInitStep0 = 2;
__host__ __device__ inline int32_t init_code(uint32_t step) {
    return step <= 0x7fffffffu - (uint32_t)kInitStep0 ? (int32_t)step + kInitStep0 : 1;
}

// Per-series statistics (lgs_diag.hip series_stats_kernel).  Series s starts at
// x + (s / gsize) * gstride + (s % gsize) * sstride, time step t at + t * tstride.
struct SeriesArgs {
    const void* x;
    int xtype;  // 0 fp64, 1 int32, 2 int64
    int64_t n_series, n, gsize, gstride, sstride, tstride;
    int64_t max_lag;  // < 0: mean / batch means only
    double window_c;  // Sokal window constant of the tau_int loop
    int64_t batch;    // > 0: batch means of this size
    double* mean;     // nullable, n_series
    double* c0;       // nullable, n_series: sum (x - mean)^2
    double* acf;      // nullable, n_series x ld_acf (lags 0..min(max_lag, n-1));
                      // null with tau set: lag blocks stop once the window closes
    int64_t ld_acf;
    double* tau;      // nullable, n_series
    double* bmeans;   // nullable, n_series x ld_b
    int64_t ld_b;
};

namespace launch {
// B z writes the kept states' moment partials (MP / MPL) on its clive path only: one
// 64-sample tile per wave (LGS_BZ_TA == 1) and the Klein launch's per-wave chunk bits
// (built by the rolled near field, not LGS_NEAR_UNROLLED; LGS_BZ_NO_CLIVE disables them)
constexpr bool bz_moments_supported() {
#if defined(LGS_BZ_NO_CLIVE) || defined(LGS_NEAR_UNROLLED) || (defined(LGS_BZ_TA) && LGS_BZ_TA != 1)
    return false;
#else
    return true;
#endif
}
// ---- diagnostics (lgs_diag.hip); xtype 0 fp64, 1 int32, 2 int64
hipError_t series_stats(const SeriesArgs& a, hipStream_t st);
// sum y y^T (d x d, both triangles) and sum y (d), y = x - shift (shift nullable),
// ADDED to G / S; x coordinate-major (d x n, ld ldz).  VALU: exact int64 for
// integer x (xtype 1 int32, 2 int64; shift int64), fp64 for xtype 0 (shift fp64).
hipError_t gram(const void* Z, int xtype, int64_t ldz, int d, int64_t n, const void* shift, void* G,
                void* S, hipStream_t st, const unsigned int* gate = nullptr);
// int8-digit path: pack y = x - shift into digit planes Ph / Pl ((d rounded up to
// 128) rows x ldp bytes, ldp = n rounded up to 64; sets kFlagI8Range when some
// |y| > 32639), then the MFMA Gram of the planes (upper block triangle + mirror:
// G must be symmetric on entry).
hipError_t gram_pack(const void* X, int xtype, bool coord_major, int64_t ldx, int d, int64_t n,
                     const long long* shift, int8_t* Ph, int8_t* Pl, int64_t ldp, unsigned int* flags,
                     hipStream_t st);
hipError_t gram_planes(const int8_t* Ph, const int8_t* Pl, int64_t ldp, int d, void* G, void* S,
                       hipStream_t st, const unsigned int* gate = nullptr);
hipError_t jump(const void* x, int xtype, int64_t n, int d, int64_t ld, double* out, hipStream_t st);
hipError_t tvd_minmax(const void* x, int xtype, int64_t n, int d, long long* mn, long long* mx,
                      unsigned int* flags, hipStream_t st);
hipError_t tvd_hist(const void* x, int xtype, int64_t n, int d, const long long* mn,
                    const long long* off, unsigned int* cnt, hipStream_t st);
hipError_t tvd_sum(const unsigned int* c1, const unsigned int* c2, const long long* off, int d,
                   int64_t n1, int64_t n2, double* out, hipStream_t st);
// binned histogram (compute_tvd's bins branch): per-column fp64 range as ordered
// int64 keys (mn / mx must start at +/- the extreme key), converted by
// hist_keys_to_f64; counts of numpy's equal-width bins ADDED to cnt (d x nb)
hipError_t hist_range(const void* x, int xtype, int64_t n, int d, long long* mn, long long* mx,
                      unsigned int* flags, hipStream_t st);
hipError_t hist_keys_to_f64(const long long* mn, const long long* mx, int d, double* lo, double* hi,
                            hipStream_t st);
hipError_t hist_counts(const void* x, int xtype, int64_t n, int d, int64_t nb, const double* edges,
                       const double* fd, unsigned long long* cnt, hipStream_t st);

// zb / ob / ib: coefficient element width in bytes (2, 4 or 8)
hipError_t klein(const KleinArgs& a, const double* R, const double* RP, const double* RC,
                 int panel, int kernel, bool wl, int zb, void* Z, hipStream_t st);
// ka: the launch's Klein arguments (certified Wang-Ling decisions recompute weights)
hipError_t accept(const AcceptArgs& a, const KleinArgs& ka, hipStream_t st);
hipError_t samplez_probe(const double* mu, const double* sig, const double* u, int64_t n,
                         int precision, int linear, int mode, const double* etab, int64_t* z, double* ln,
                         hipStream_t st);
hipError_t log_density(const KleinArgs& a, const double* R, const void* Z, int zb, double* out,
                       hipStream_t st);
// moments of the proposal store + (fsel non-null) the chains' final states into zs
// abort (nullable) below: the kernel returns at once when *abort & kAbortMask
hipError_t moments_final(const void* Z, int zb, int64_t ldz, const int32_t* cnt, int64_t n, int64_t T,
                         const int64_t* fsel, int d, unsigned long long* mom, void* zs, int ob,
                         int zs_cm, int64_t nc, hipStream_t st, const unsigned int* abort,
                         const uint8_t* znz = nullptr, int64_t zlanes = 0, int zshift = 0,
                         const unsigned int* need = nullptr);
hipError_t moments_carry(const void* zs, int zb, int coord_major, int64_t nc, int d,
                         const int32_t* cc, unsigned long long* mom, hipStream_t st,
                         const unsigned int* abort = nullptr, const unsigned int* need = nullptr);
hipError_t gather_z(const void* Z, int zb, int64_t ldz, const int64_t* sel, int64_t nq,
                    int64_t q_per_chain, const void* zs, int ob, int zs_coord_major, int64_t nc,
                    int d, void* out, int out_coord_major, hipStream_t st,
                    const unsigned int* abort = nullptr);
// initial IMHK draws decided on the device: uninit_scan sets *any when some
// init[c] == 0; init_apply (gated by *any, abortable) gives each such chain the
// proposal of column c of Z (ld nc) and its log weight LW[c], and marks it initialised
hipError_t uninit_scan(const int32_t* init, int64_t nc, unsigned int* any, hipStream_t st);
// (flags: the context's flag words; init_apply also checkpoints the resolved count)
hipError_t init_apply(const void* Z, int zb, int32_t* init, int64_t nc, int d, const double* LW, void* zs,
                      int ob, int zs_cm, double* lws, unsigned int* flags, hipStream_t st);
hipError_t transpose_out(const void* Z, int zb, int64_t ldz, int64_t n, int d, void* out, int ob,
                         hipStream_t st);
hipError_t to_coord_major(const void* in, int ib, int64_t n, int d, void* Z, int zb, int64_t ldz,
                          hipStream_t st);
// V row of sample s: (s / rb) * rstride + roff + s % rb (rb = n, rstride = roff = 0: row s)
hipError_t bz(const void* Z, int zb, int64_t ldz, const int64_t* sel, const double* BT, int d,
              int64_t n, double* V, int64_t ldv, int64_t rb, int64_t rstride, int64_t roff,
              hipStream_t st, const unsigned int* abort = nullptr, const unsigned int* need = nullptr);
hipError_t bz_i8(const void* Z, int zb, int64_t ldz, const int64_t* sel, const int* kchunk,
                 const int* koff, const int8_t* Bd1, const int8_t* Bd0, int dc, int d, int64_t n,
                 double* V, int64_t ldv, int64_t rb, int64_t rstride, int64_t roff,
                 unsigned int* flags, const int16_t* h16, int64_t h16_lanes, int64_t hcols,
                 hipStream_t st, const unsigned int* abort = nullptr, const uint8_t* znz = nullptr,
                 const unsigned int* clive = nullptr, int64_t clive_ld = 0, double* VNP = nullptr,
                 int64_t vn_n = 0, unsigned long long* MP = nullptr, int64_t mp_ld = 0,
                 unsigned int* MPL = nullptr);
// moments of the kept states from bz_i8's per-(tile, coordinate) partials MP (packed
// sum over the tile's 64 rows of z^2 * 2^24 + z + 32768; MPL: the tile's live-chunk
// words, (d + 2047) / 2048 per tile), added to mom (2d); returns at once when *flags has
// kFlagI8Range (the gated moments pass replaces it then)
hipError_t bz_moments_reduce(const unsigned long long* MP, const unsigned int* MPL, int64_t ntiles, int64_t mp_ld,
                             int d,
                             unsigned long long* mom, const unsigned int* flags, hipStream_t st,
                             const unsigned int* abort);
// the chains' states after a block from the int16 history of the block's Klein launch:
// zs[c] = proposal fsel[c] (kept as is when fsel[c] < 0); history [d / 16][lanes][16] of z + 128
hipError_t final_h16(const int16_t* h16, int64_t lanes, const int64_t* fsel, int64_t nc, int d, void* zs,
                     int ob, int zs_cm, hipStream_t st, const unsigned int* abort);
// VNP (nullable, 2 ceil(d / 128) x vn_n): per-(half coordinate tile, row) partial sums of
// ||v||^2 of rows q < vn_n (bz_i8), summed per row into VN by vnorm2_reduce (n = vn_n)
hipError_t vnorm2_reduce(const double* VNP, int d, int64_t n, int64_t rb, int64_t rstride, int64_t roff,
                         double* VN, hipStream_t st, const unsigned int* abort = nullptr);
// scalar functionals of kept states: coefficient k of selection q, and
// ||v||^2 of the rows of V (row index (q / rb) * rstride + roff + q % rb in both)
// lag-L sums of nc per-chain series (int64, or fp64 scaled by scale), T new values each
// (row stride ldx), continued through ring (nc x L); sums (L + 2: lags 0..L, then sum x)
// added to; P scratch of (L + 2) nc values
hipError_t lag_update(const void* X, int is_f64, int64_t ldx, int64_t nc, int64_t Tn, int L, double scale,
                      void* ring, void* sums, void* P, hipStream_t st, const unsigned int* abort = nullptr);
hipError_t coord_gather(const void* Z, int zb, int64_t ldz, const int64_t* sel, int64_t nq, int64_t q_per_chain,
                        const void* zs, int ob, int zs_coord_major, int64_t nc, int d, int k, int64_t* out,
                        int64_t rb, int64_t rstride, int64_t roff, hipStream_t st, const unsigned int* abort);
hipError_t vnorm2_rows(const double* V, int d, int64_t n, int64_t rb, int64_t rstride, int64_t roff, double* VN,
                       hipStream_t st, const unsigned int* abort = nullptr, const unsigned int* need = nullptr);
// ---- decoding
// V (row-major n x d) = rows s: sum_c MT[c][r] X[c][s], X coordinate-major fp64 (fp64 MFMA)
hipError_t gemm_f64(const double* X, int64_t ldx, const double* MT, int d, int64_t n, double* V,
                    hipStream_t st);
hipError_t nearest_plane(int d, int64_t n, int panel, const double* RP, const double* RC,
                         const double* rii, const double* CP, int64_t ldc, int zb, void* Z, int64_t ldz,
                         unsigned int* flags, hipStream_t st);
hipError_t round_coeffs(const double* W, int64_t ldw, int d, int64_t n, int zb, void* Z, int64_t ldz,
                        unsigned int* flags, hipStream_t st);
hipError_t check_range16(const void* zs, int ob, int64_t count, unsigned int* flags, hipStream_t st);
// (a value that does not fit a 16-bit store sets kFlagCarry16 in *flags)
hipError_t carry_cols(const void* zs, int ob, int zs_coord_major, int64_t nc, int d, void* Z, int zb,
                      int64_t ldz, int64_t col0, hipStream_t st, unsigned int* flags = nullptr);
}  // namespace launch
}  // namespace lgs
