// gs_device.hpp — the CDNA4 (gfx950) device code of the GMG V-cycle and its launch plans: point
// formulas, the stencil / restriction / prolongation / coarse-cycle kernels and the host-side planning
// helpers. Included by gs_kernels.hip (the product library, include/gpusolve_hip.h) and by gs_diag.hip
// (libgpusolve_diag.so: tuning variants, bandwidth probes and the measured-and-rejected k_prr, which only
// tools/, tests/ and bench.py's measured-ceiling leg load; include/gpusolve_diag.h). Internal linkage.
//
// Numerics follow the reference CPU backend operator by operator (src/cpu/CpuSolver.cpp,
// src/cpu/NewtonSolver.cpp, src/cpu/CpuGridData.cpp of Bricktricker/gpu-solve): every expression
// keeps the reference's evaluation order and the libraries are built with -ffp-contract=off, so in
// LINEAR mode every field is bit-identical to the CPU path; only the l2-norm summation order
// (deterministic here: fixed per-block partials + fixed-order finish) and, in the non-linear
// modes, ocml's exp vs glibc's exp (<= 1 ulp) differ.
//
// Layout: x unit-stride, z slowest (include/gpusolve_hip.h), so Z-slabs are contiguous planes and
// a wave64 row load along x is one coalesced 1 KiB (dwordx4 per lane) access.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include <cmath>
#include <stdint.h>
#include <stdlib.h>

#include <map>
#include <mutex>
#include <utility>

#include "gpusolve_hip.h"

// Timing-only experiment builds (tools/exp_builds.sh; never the product, results are wrong):
//   GS_EXP_NOBAR  the pair's and k_rr2's per-plane LDS barriers removed (what the lock-step costs)
//   GS_EXP_NOEXP  exp(x) replaced by one multiplication (what the exponentials cost)
//   GS_EXP_NODIV  NEWTON's r / den replaced by a multiplication (what the divisions cost)
//   GS_EXP_EFIELD k_tb2y's NEWTON sweep-1 rows load E = exp(w) from a second field instead of evaluating it
//                 (the field lies gs_exp_set_efoff(n) elements past newtonV; tools/newton_kprobe.py sets it)
// Alternative-arithmetic builds (A/B only; correct results, not the product's choice):
//   GS_EXP_NB_IEEE   GS_NEWTON_B's Jacobi quotient as the IEEE division instead of nb_quot (r05p)
#ifdef GS_EXP_NOEXP
#define exp(x) ((x) * 1.0000001)
#endif
#ifdef GS_EXP_NOBAR
#define GS_LDS_BARRIER() __builtin_amdgcn_s_waitcnt(0xc07f)
#else
#define GS_LDS_BARRIER()                                                                                               \
    do {                                                                                                               \
        __builtin_amdgcn_s_waitcnt(0xc07f);                                                                            \
        __builtin_amdgcn_s_barrier();                                                                                  \
    } while (0)
#endif

namespace {

constexpr int WAVE = 64;

// NEWTON's two forms (include/gpusolve_hip.h): GS_NEWTON reads newtonV as w, GS_NEWTON_B reads the precomputed
// linearisation factor B = gamma (1 + newtonV) exp(newtonV) (gs_newton_bfac) as w. Both carry a w operand.
constexpr bool newtonish(int m) { return m == GS_NEWTON || m == GS_NEWTON_B; }
// GS_NEWTON_G (the first Newton iteration: B = gamma everywhere) launches the GS_NEWTON_B kernels with Coef::bconst
constexpr int base_mode(int m) { return m == GS_NEWTON_G ? GS_NEWTON_B : m; }

// compile-time / run-time booleans for code specialised per wave (BoolC) or selected per use (RtBool)
template <bool B>
struct BoolC {
    __device__ static constexpr bool get() { return B; }
};
struct RtBool {
    bool b;
    __device__ bool get() const { return b; }
};

// ---------------------------------------------------------------------------------------------
// Stencil coefficients by value (they land in SGPRs).
struct Coef {
    double s[7];
    double hh;     // h*h
    double omega;
    double gamma;
    double alpha;  // h*h / s0          (CpuSolver.cpp:145)
    double preFac; // s0 / (h*h)        (CpuSolver.cpp:144)
    int fastdiv;   // 2^-120 <= hh <= 1: div_hh may take its 3-operation path
    int unit;      // s[1..6] == -1 and |s[0]| >= 1: the unit-neighbour stencil sum applies (stencil_sum<true>)
    int swz;       // column-block pairs: x-waves of the mirrored row rotated by two (GS_XH_SWIZZLE)
    int zq;        // every s[i] finite and hh a positive normal number: the stencil sum of an identically zero
                   // iterate over hh is exactly +0 (each s[i] * 0 is a signed zero, +0 plus a signed zero is
                   // +0, +0 / hh is +0), so zero-iterate sweeps take q = +0 without evaluating it
    int bconst;     // GS_NEWTON_B with B = gamma at every point (the first Newton iteration's factor): the pair and
                    // k_rr2 take k.gamma instead of loading w (which still holds gamma for every other kernel)
    int64_t off[7]; // generic kernel: linear element offsets of the 7 entries
#ifdef GS_EXP_EFIELD
    int64_t efoff;
#endif
};

bool canonical_order(const gs_stencil* S)
{
    static const int cx[7] = {0, 1, -1, 0, 0, 0, 0};
    static const int cy[7] = {0, 0, 0, 1, -1, 0, 0};
    static const int cz[7] = {0, 0, 0, 0, 0, 1, -1};
    for (int i = 0; i < 7; i++)
        if (S->ox[i] != cx[i] || S->oy[i] != cy[i] || S->oz[i] != cz[i]) return false;
    return true;
}

bool valid_stencil(const gs_stencil* S)
{
    for (int i = 0; i < 7; i++)
        if (S->ox[i] < -1 || S->ox[i] > 1 || S->oy[i] < -1 || S->oy[i] > 1 || S->oz[i] < -1 || S->oz[i] > 1)
            return false;
    return true;
}

// A/B switches of the launch plans, read ONCE when the library is loaded (a namespace-scope object,
// initialised at load time: no getenv is reachable from a launch). Defaults are the measured choices
// (DESIGN.md §9); the switches serve tools/ A/B runs and the tests that pin every alternative path:
//   GS_NO_UNIT_STENCIL   the general 14-operation stencil sum instead of the unit-neighbour form
//   GS_TBX_PFD=1         column-block pairs at one plane step of prefetch (default 2)
//   GS_PAIR_XH=0         rows > 512 points on k_tb2's one-y-wave shape instead of column blocks
//   GS_FIT_ROUNDS=0      no round-fitted chunk lengths for the zero-iterate pairs
//   GS_SLAB_ZC=n         z-chunk (planes; even, >= 2) of pair launches past a slab's first plane
//   GS_PAIR_ZC=n         z-chunk of pair launches from a level's first plane (>= 2^26 points)
//   GS_PAIR_MIN_BLOCKS=n blocks of 4-plane chunks from which a level smooths in pairs (default 128)
//   GS_PAIR_BIG_CHUNKS=0 64-plane chunks on >= 2^26-point levels
//   GS_PAIR_ONE_ROUND=0  no one-round / four-round chunking on >= 2^26-point levels
//   GS_RR_LDS            residual + restriction through the LDS kernel (k_resrestrict) only
//   GS_RR_NR=1|2         coarse rows per k_rr2 block (default: 2 on LINEAR levels of >= 2^26 points)
//   GS_RR_NTU=0|1        k_rr2 non-temporal loads never / on two-row blocks only (default 2: every block, r05w)
//   GS_RR_REVERSE=0|1    k_rr2 z-chunks in ascending (0) or descending (1, default: r04e, -1% on 512^3) order
//   GS_NO_ZERO_Q         zero-iterate sweeps evaluate the stencil of their zeros instead of taking q = +0
//   GS_XH_SWIZZLE=0|1    column-block pairs: the mirrored row's x-waves rotated by two (1, default) or not (0)
//   GS_MID_ZC=n          z-chunk of pair launches over whole levels of < 2^26 points (A/B)
//   GS_RR_ZC=n           z-chunk (coarse planes) of k_rr2 launches from fine levels of < 2^26 points (A/B)
//   GS_RR_ZC_BIG=n       the same for fine levels of >= 2^26 points (A/B)
//   GS_PAIR_ONE_ROUND_MID=1 LINEAR pair launches over levels of 2^24 .. 2^26 points in one round of blocks (A/B)
//   GS_RB_ZC=n           z-chunk of the one-point passes (k_rb sweeps / residuals, the Newton update pass) (A/B)
//   GS_NEWTON_XH=0       NEWTON plain pairs on rows of 513-1024 points through k_tb2 instead of column blocks (A/B)
//   GS_SPEC_CACHED=1     pairs with norm partials store through the caches, not non-temporally (A/B)
//   GS_RR_NG=2           k_rr2 with two groups of coarse rows per block (default 1: measured faster, r05b)
//   GS_PAIR_FX=0         LINEAR plain pairs always through the instance with per-lane range selects (A/B, r06)
struct Knobs {
    bool unitStencil, tbxPfd2, pairXh, fitRounds, bigChunks, oneRound, rrLds, zeroQ, newtonXh, specCached;
    int xhSwizzle, midZc, rrZc, rrZcBig, oneRoundMid, rbZc;
    int slabZc, pairZc, rrNr, rrNtu, rrReverse, rrNg, rrDma;
    bool pairFx;
    int64_t pairMinBlocks;
    static int num(const char* name, int dflt)
    {
        const char* e = getenv(name);
        return e && *e ? atoi(e) : dflt;
    }
    Knobs()
        : unitStencil(getenv("GS_NO_UNIT_STENCIL") == nullptr), tbxPfd2(num("GS_TBX_PFD", 2) != 1),
          pairXh(num("GS_PAIR_XH", 1) != 0), fitRounds(num("GS_FIT_ROUNDS", 1) != 0),
          bigChunks(num("GS_PAIR_BIG_CHUNKS", 1) != 0), oneRound(num("GS_PAIR_ONE_ROUND", 1) != 0),
          rrLds(getenv("GS_RR_LDS") != nullptr), zeroQ(getenv("GS_NO_ZERO_Q") == nullptr),
          newtonXh(num("GS_NEWTON_XH", 1) != 0), specCached(num("GS_SPEC_CACHED", 0) != 0),
          xhSwizzle(num("GS_XH_SWIZZLE", 1)), midZc(num("GS_MID_ZC", 0)), rrZc(num("GS_RR_ZC", 0)), rrZcBig(num("GS_RR_ZC_BIG", 0)), oneRoundMid(num("GS_PAIR_ONE_ROUND_MID", 0)), rbZc(num("GS_RB_ZC", 0)), slabZc(num("GS_SLAB_ZC", 0)), pairZc(num("GS_PAIR_ZC", 0)),
          rrNr(num("GS_RR_NR", 0)), rrNtu(num("GS_RR_NTU", 2)), rrReverse(num("GS_RR_REVERSE", 1)), rrNg(num("GS_RR_NG", 0)), rrDma(num("GS_RR_DMA", 0)),
          pairFx(num("GS_PAIR_FX", 1) != 0),
          pairMinBlocks(num("GS_PAIR_MIN_BLOCKS", 128))
    {
    }
};
const Knobs kKnobs;

#ifdef GS_EXP_EFIELD
int64_t gs_exp_efoff = 0; // set by gs_exp_set_efoff (gs_kernels.hip, this build only)
#endif

Coef make_coef(const gs_stencil* S, const gs_level* L, double omega, double gamma, int bconst = 0)
{
    Coef k;
    for (int i = 0; i < 7; i++) {
        k.s[i] = S->s[i];
        k.off[i] = S->ox[i] + S->oy[i] * L->ldy + S->oz[i] * L->ldz;
    }
    k.hh = L->h * L->h;
    k.omega = omega;
    k.gamma = gamma;
    k.alpha = k.hh / S->s[0];
    k.preFac = S->s[0] / k.hh;
    k.fastdiv = k.hh >= 0x1p-120 && k.hh <= 1.0;
    k.unit = kKnobs.unitStencil && (S->s[0] >= 1.0 || S->s[0] <= -1.0);
    for (int i = 1; i < 7; i++) k.unit = k.unit && S->s[i] == -1.0;
    k.swz = kKnobs.xhSwizzle;
    k.zq = kKnobs.zeroQ && std::isnormal(k.hh) && k.hh > 0.0;
    for (int i = 0; i < 7; i++) k.zq = k.zq && std::isfinite(S->s[i]);
    k.bconst = bconst;
#ifdef GS_EXP_EFIELD
    k.efoff = gs_exp_efoff;
#endif
    return k;
}

// ---------------------------------------------------------------------------------------------
// Point formulas (reference evaluation order; built with -ffp-contract=off).

// s / hh, bit-identical to the compiler's IEEE division, in 3 FP64 operations instead of ~11.
// The gfx950 division sequence is: D = div_scale(hh), y = rcp(D) refined by two Newton steps,
// N = div_scale(s), q = N*y, r = fma(-D, q, N), q' = div_fmas(r, y, q), div_fixup(q', hh, s). When
// neither operand is scaled (s and hh normal, s != 0, exponent(s) - exponent(hh) < 768, the quotient
// normal and exponent(s) > 53) div_scale returns its operand, div_fmas is a plain fma and div_fixup
// returns q' — and y depends on hh alone, so it is loop-invariant. The fast path is taken for
// 2^-899 <= |s| < 2^601 with the host guaranteeing 2^-120 <= hh <= 1 (Coef::fastdiv); anything
// else (zero, denormals, inf/nan, extreme magnitudes) takes the ordinary division.
__device__ __forceinline__ double hh_recip(double hh)
{
    const double y0 = __builtin_amdgcn_rcp(hh);
    const double y1 = __builtin_fma(y0, __builtin_fma(-hh, y0, 1.0), y0);
    return __builtin_fma(y1, __builtin_fma(-hh, y1, 1.0), y1);
}

__device__ __forceinline__ double div_hh(const Coef& k, double s)
{
    const unsigned e = ((unsigned)__double2hiint(s) >> 20) & 0x7ffu; // biased exponent
    if (k.fastdiv && e - 124u < 1500u) {                              // 124 <= e <= 1623
        const double y = hh_recip(k.hh);
        const double q = s * y;
        const double r = __builtin_fma(-k.hh, q, s);
        return __builtin_fma(r, y, q);
    }
    return s / k.hh;
}

// The same division for N values at once: the operand-range test of every value is combined first
// and ONE branch picks the 3-operation path for all N (or the IEEE division for all N when any value
// is outside the range), so a sweep over several rows has one exec branch instead of one per point
// and the scheduler can interleave the rows' arithmetic.
__device__ __forceinline__ bool div_hh_fast_ok(double s)
{
    const unsigned e = ((unsigned)__double2hiint(s) >> 20) & 0x7ffu;
    return e - 124u < 1500u;
}
template <int N>
__device__ __forceinline__ void div_hh_n(const Coef& k, double (&s)[N])
{
    bool ok = k.fastdiv;
#pragma unroll
    for (int i = 0; i < N; i++) ok &= div_hh_fast_ok(s[i]);
    if (ok) {
        const double y = hh_recip(k.hh);
#pragma unroll
        for (int i = 0; i < N; i++) {
            const double q = s[i] * y;
            const double r = __builtin_fma(-k.hh, q, s[i]);
            s[i] = __builtin_fma(r, y, q);
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; i++) s[i] = s[i] / k.hh;
    }
}

// one row's two points: batched, except in GS_NEWTON mode whose kernels run at the VGPR limit (the batch
// keeps both sums live across the branch). GS_NEWTON_B's pairs have the room since r05: batched, NEWTON_B pair
// 0.840-0.853 vs 0.872-0.885 ms, prolongation pair 0.924-0.930 vs 0.964-0.975 ms, Newton iteration -0.8 ms (r05r)
template <int MODE>
__device__ __forceinline__ void div_hh_row(const Coef& k, double (&q)[2])
{
    if (MODE == GS_NEWTON) {
        q[0] = div_hh(k, q[0]);
        q[1] = div_hh(k, q[1]);
    } else {
        div_hh_n(k, q);
    }
}

// stencil sum in config order (before the division by h^2) — CpuSolver.cpp:56-62.
// UN (Coef::unit: the six neighbour weights are exactly -1, |s0| >= 1 — every reference config): the
// same value in 7 instead of 14 operations, bit for bit. s += (-1) * x is s - x exactly (the product
// by -1 is a sign flip, and IEEE subtraction is the addition of the negation), and the first term
// 0.0 + s0 * c equals fma(s0, c, 0.0): both round the product once and add an exact zero, and with
// |s0| >= 1 a non-zero product never underflows to a signed zero (the one case where they differ).
template <bool UN = false>
__device__ __forceinline__ double stencil_sum(const Coef& k, double c, double xp, double xm, double yp, double ym,
                                              double zp, double zm)
{
    if constexpr (UN) {
        double s = __builtin_fma(k.s[0], c, 0.0);
        s = s - xp;
        s = s - xm;
        s = s - yp;
        s = s - ym;
        s = s - zp;
        s = s - zm;
        return s;
    }
    double s = 0.0;
    s += k.s[0] * c;
    s += k.s[1] * xp;
    s += k.s[2] * xm;
    s += k.s[3] * yp;
    s += k.s[4] * ym;
    s += k.s[5] * zp;
    s += k.s[6] * zm;
    return s;
}

// the non-linear term added after the division — CpuSolver.cpp:63-76
template <int MODE>
__device__ __forceinline__ double op_finish(const Coef& k, double q, double c, double w)
{
    if (MODE == GS_NEWTON) {
        const double ew = exp(w);
        q += k.gamma * (1 + w) * c * ew;
    } else if (MODE == GS_NEWTON_B) {
        q += w * c; // w = B = gamma (1 + newtonV) exp(newtonV)
    } else if (MODE == GS_NONLINEAR) {
        const double ev = exp(c);
        const double nl = k.gamma * c * ev;
        q += nl;
    }
    return q;
}

// stencil sum in config order, then /h^2 and the non-linear term  — CpuSolver.cpp:56-76
template <int MODE, bool UN = false>
__device__ __forceinline__ double op_value(const Coef& k, double c, double xp, double xm, double yp, double ym,
                                           double zp, double zm, double w)
{
    double s = stencil_sum<UN>(k, c, xp, xm, yp, ym, zp, zm);
    s = div_hh(k, s);
    return op_finish<MODE>(k, s, c, w);
}

// GS_NEWTON_B's Jacobi quotient r / den (den = preFac + B, the reference's denominator bit for bit): r times den's
// reciprocal refined by two Newton steps (the reciprocal the IEEE division sequence forms, see div_hh), without the
// division's final correction, scaling and fix-up: 7 FP64 operations instead of ~11, branch-free, and within 1 ulp
// of r / den (tests/test_gpu_newton_b.py::test_nb_quotient_ulps: 26 % of the quotients differ, by one ulp). NEWTON's
// parity is a tolerance — 1e-6 relative on the residual norms (north_star), 1e-9 / 1e-10 in the tests — and its exp
// already differs by an ulp between ocml and glibc. A denominator above 2^1000 (inf included) is clamped there so the
// reciprocal stays normal: r / inf comes out below |r| 2^-999 instead of 0; NaN stays NaN, den = 0 gives NaN where the
// IEEE quotient is inf — both non-finite. Per 512^3 launch: pair 0.871-0.873 vs 0.897-0.914 ms, prolongation pair
// 0.960-0.965 vs 0.989-0.997 ms; Newton iteration -0.5 ms (r05p, profiles/r05/r05p_newton_b_quotient_ab.txt; one
// Newton step only: 18 ulp, 1 % faster; a range branch around it: r05o). GS_EXP_NB_IEEE: the IEEE division (A/B).
// The clamp is symmetric (r06): B = gamma (1 + w) e^w is negative for w < -1, so preFac + B can be negative; a
// denominator of magnitude above 2^1000 (-inf included) keeps its sign. Denominators of magnitude 2^-1000 .. 2^1000
// of either sign stay within the 1 ulp (test_nb_quotient_ulps); below that the reciprocal overflows to inf, where the
// IEEE quotient may still be finite (a point whose denominator cancels to ~1e-301 has left the contract anyway).
__device__ __forceinline__ double nb_recip(double den)
{
    const double d = __builtin_fabs(den) > 0x1p1000 ? __builtin_copysign(0x1p1000, den) : den;
    return hh_recip(d);
}
__device__ __forceinline__ double nb_quot(double r, double den)
{
#ifdef GS_EXP_NB_IEEE
    return r / den;
#else
    return r * nb_recip(den);
#endif
}

// Jacobi point update from the old value and its residual — CpuSolver.cpp:157-171
template <int MODE>
__device__ __forceinline__ double jacobi_update(const Coef& k, double v, double r, double w)
{
    if (MODE == GS_LINEAR) return v + k.omega * (k.alpha * r);
    if (MODE == GS_NEWTON_B) return v + k.omega * nb_quot(r, k.preFac + w); // preFac + B: the reference's den
    const double u = (MODE == GS_NONLINEAR) ? v : w;
    const double eu = exp(u);
    const double den = k.preFac + k.gamma * (1 + u) * eu;
    return v + k.omega * (r / den);
}

// NEWTON's linearisation terms of a point, A = gamma (1 + w) and E = exp(w), computed ONCE per point
// and pass and shared by the operator and the update of both sweeps of a fused pair: bit-identical to
// op_finish / jacobi_update, whose reference expressions evaluate gamma * (1 + w) first and multiply
// by exp(w) last (CpuSolver.cpp:63-66, :157-171).
__device__ __forceinline__ double newton_op(double q, double c, double A, double E) { return q + A * c * E; }
template <int MODE>
__device__ __forceinline__ double newton_update(const Coef& k, double v, double r, double A, double E)
{
    const double den = k.preFac + A * E;
    if constexpr (MODE == GS_NEWTON_B) return v + k.omega * nb_quot(r, den); // (E = 1: den = preFac + B exactly)
#ifdef GS_EXP_NODIV
    return v + k.omega * (r * den);
#else
    return v + k.omega * (r / den);
#endif
}

// GS_NEWTON_B's linearisation factor of a point, b = gamma (1 + w) exp(w), evaluated as the reference's Jacobi
// denominator evaluates its product, (gamma * (1 + w)) * exp(w) (CpuSolver.cpp:166-172)
__device__ __forceinline__ double bfac_of(double gamma, double w) { return gamma * (1 + w) * exp(w); }

// A and E of a point from its w operand: GS_NEWTON_B's w is B itself, so A = B and E = 1 (A * c * E = B * c and
// preFac + A * E = preFac + B exactly: the products by 1.0 fold away)
template <int MODE>
__device__ __forceinline__ double newton_A(const Coef& k, double w)
{
    return MODE == GS_NEWTON_B ? w : k.gamma * (1 + w);
}
template <int MODE>
__device__ __forceinline__ double newton_E(double w)
{
    return MODE == GS_NEWTON_B ? 1.0 : exp(w);
}

__device__ __forceinline__ double wave_sum(double x)
{
#pragma unroll
    for (int o = WAVE / 2; o > 0; o >>= 1) x += __shfl_down(x, o, WAVE);
    return x;
}

// Block-wide fixed-order sum of nw <= NWAVES waves (default: all); result valid in thread 0.
template <int NWAVES>
__device__ __forceinline__ double block_sum(double x, double* lds, int nw = NWAVES)
{
    const int tid = threadIdx.x + threadIdx.y * blockDim.x;
    x = wave_sum(x);
    if ((tid & (WAVE - 1)) == 0) lds[tid / WAVE] = x;
    __syncthreads();
    double t = 0.0;
    if (tid == 0) {
#pragma unroll
        for (int i = 0; i < NWAVES; i++)
            if (i < nw) t += lds[i];
    }
    return t;
}

// ---------------------------------------------------------------------------------------------
// Stencil passes come in three kinds:
//   KIND 0: Jacobi sweep         out = v_new (partials: sum r^2 of the input's residual, nullable)
//   KIND 1: residual             out = r (nullable), partials = per-block sum r^2 (nullable)
//   KIND 2: FAS coarse operator  out = A(u) (ADD=false) or out += A(u) (ADD=true)
// ---------------------------------------------------------------------------------------------
// Register-blocked z-march ("rb"): each lane owns 2 consecutive x-points (one dwordx4) of RY
// consecutive y-rows, a wave owns a 128 x RY tile, W waves stack in y, the block walks ZC planes.
//  - y-neighbours come from the lane's own registers (plus 2 halo rows per wave and plane),
//  - x-neighbours from the adjacent lane by a DPP wave shift (wave_shr:1 / wave_shl:1); the two
//    tile-edge values per row are wave-uniform scalar loads,
//  - z-neighbours are the previous / next plane held in registers,
//  - every load of plane z+1 (next-next v rows, halo rows, f, edges) is issued before plane z is
//    computed, so a full plane of HBM traffic is in flight behind the arithmetic.
// Loads use a clamped column min(x, nx+1); a pair load there reads one element past the padded
// row, which the allocation recipe of gs_field_layout (+32 elements) keeps in bounds.
template <bool DPP>
__device__ __forceinline__ double lane_from_left(double src, double edge)
{
    // lane i <- src of lane i-1; lane 0 <- edge
    if (DPP) {
        const long long s = __double_as_longlong(src), e = __double_as_longlong(edge);
        const int lo = __builtin_amdgcn_update_dpp((int)e, (int)s, 0x138, 0xf, 0xf, false);
        const int hi = __builtin_amdgcn_update_dpp((int)(e >> 32), (int)(s >> 32), 0x138, 0xf, 0xf, false);
        return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
    } else {
        const double t = __shfl_up(src, 1, WAVE);
        return (threadIdx.x & (WAVE - 1)) == 0 ? edge : t;
    }
}

template <bool DPP>
__device__ __forceinline__ double lane_from_right(double src, double edge)
{
    // lane i <- src of lane i+1; lane 63 <- edge
    if (DPP) {
        const long long s = __double_as_longlong(src), e = __double_as_longlong(edge);
        const int lo = __builtin_amdgcn_update_dpp((int)e, (int)s, 0x130, 0xf, 0xf, false);
        const int hi = __builtin_amdgcn_update_dpp((int)(e >> 32), (int)(s >> 32), 0x130, 0xf, 0xf, false);
        return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
    } else {
        const double t = __shfl_down(src, 1, WAVE);
        return (threadIdx.x & (WAVE - 1)) == WAVE - 1 ? edge : t;
    }
}

// a value every lane holds identically (an LDS broadcast read), moved to SGPRs
__device__ __forceinline__ double uniform_d(double x)
{
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readfirstlane((int)b), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double2 ld2(const double* __restrict__ p) { return *reinterpret_cast<const double2*>(p); }

typedef double dv2 __attribute__((ext_vector_type(2)));
// streamed-once operands (f, the output) optionally bypass the caches' retention (nt)
template <bool NT>
__device__ __forceinline__ double2 ld2s(const double* __restrict__ p)
{
    if (NT) {
        const dv2 t = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(p));
        return make_double2(t.x, t.y);
    }
    return ld2(p);
}
template <bool NT>
__device__ __forceinline__ void st2s(double* __restrict__ p, double a, double b)
{
    if (NT) {
        const dv2 t = {a, b};
        __builtin_nontemporal_store(t, reinterpret_cast<dv2*>(p));
    } else {
        *reinterpret_cast<double2*>(p) = make_double2(a, b);
    }
}

// Loads of the iterate; ZV: the iterate is identically zero (a coarse level's first sweep after
// the reference's v = 0) and is not read at all. Multiplying the literal zeros keeps the arithmetic,
// and so every bit of the result, that of loaded zeros (no fast-math folding).
template <bool ZV, bool NT = false>
__device__ __forceinline__ double2 ldv2(const double* __restrict__ p)
{
    if (ZV) return make_double2(0.0, 0.0);
    return ld2s<NT>(p);
}
template <bool ZV>
__device__ __forceinline__ double ldv1(const double* __restrict__ p)
{
    return ZV ? 0.0 : *p;
}

// Bijective XCD-aware tile order (cdna_hip_programming.md T1): hardware block b runs on XCD b % 8;
// give each XCD a contiguous run of tiles so y-neighbour tiles share an L2 while they run.
__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t nb)
{
    const int64_t q = nb / 8, r = nb % 8, x = b % 8, k = b / 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

template <int MODE, int KIND, bool ADD, int RY, int W, bool DPP, bool NT = false, bool XCD = false, bool NTV = false,
          bool ZV = false, bool UN = false>
__global__ __launch_bounds__(WAVE* W) void k_rb(Coef k, const double* __restrict__ v, const double* __restrict__ f,
                                                 const double* __restrict__ w, double* __restrict__ out,
                                                 double* __restrict__ partials, int nx, int ny, int nz, int64_t ldy,
                                                 int64_t ldz, int ZC)
{
    __shared__ double red[W];
    const int lane = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.y);
    int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    int64_t tile = blockIdx.x + gridDim.x * ((int64_t)blockIdx.y + gridDim.y * (int64_t)blockIdx.z);
    if (XCD) {
        const int nbx = (nx + 2 * WAVE - 1) / (2 * WAVE), nby = (ny + RY * W - 1) / (RY * W);
        tile = xcd_tile(blockIdx.x, gridDim.x);
        bx = (int)(tile % nbx);
        by = (int)((tile / nbx) % nby);
        bz = (int)(tile / ((int64_t)nbx * nby));
    }
    const int x0 = 1 + bx * (2 * WAVE);
    const int x = x0 + 2 * lane;
    const int xl = min(x, nx + 1);
    const int y0 = 1 + (by * W + wv) * RY;
    const int zb = 1 + bz * ZC;
    const int ze = min(zb + ZC - 1, nz);
    const int xle = x0 - 1;
    const int xre = min(x0 + 2 * WAVE, nx + 1);
    const bool okx0 = x <= nx, okx1 = x + 1 <= nx;
    const double* fin = (KIND == 2) ? out : f;

    int64_t roff[RY + 2]; // rows y0-1 .. y0+RY (clamped into the padded range)
#pragma unroll
    for (int r = 0; r < RY + 2; r++) roff[r] = (int64_t)min(y0 - 1 + r, ny + 1) * ldy;

    // Planes z-1 (P) and z (C) of the wave's rows live in registers. Everything of plane z+1 (its
    // halo rows, f, w, tile edges) and the v rows of plane z+2 is loaded into slot ph of a two-slot
    // ring while plane z is computed from the other slot, and only moved out after it was consumed:
    // a load's destination is never copied before its first use, so its wait lands one full plane
    // of arithmetic after the issue (the loop is unrolled by two to make the slot index static).
    double2 P[RY], C[RY], NL[2][RY], FL[2][RY], WL[2][RY], HL[2][2];
    double EL[2][RY], ER[2][RY];
    double sumsq = 0.0;
    // slot s <- plane z1's halo rows, f, w, edges and plane z2's v rows (plane offsets)
    auto load_slot = [&](const int s, const int64_t z1, const int64_t z2) {
#pragma unroll
        for (int r = 0; r < RY; r++) {
            NL[s][r] = ldv2<ZV, NTV>(v + xl + roff[r + 1] + z2);
            if (KIND != 2 || ADD) FL[s][r] = ld2s<NT>(fin + xl + roff[r + 1] + z1);
            if (newtonish(MODE)) WL[s][r] = ld2(w + xl + roff[r + 1] + z1);
            EL[s][r] = ldv1<ZV>(v + xle + roff[r + 1] + z1);
            ER[s][r] = ldv1<ZV>(v + xre + roff[r + 1] + z1);
        }
        HL[s][0] = ldv2<ZV>(v + xl + roff[0] + z1);
        HL[s][1] = ldv2<ZV>(v + xl + roff[RY + 1] + z1);
    };
    if (zb <= ze) {
        const int64_t zo = (int64_t)zb * ldz;
#pragma unroll
        for (int r = 0; r < RY; r++) {
            P[r] = ldv2<ZV>(v + xl + roff[r + 1] + zo - ldz);
            C[r] = ldv2<ZV>(v + xl + roff[r + 1] + zo);
        }
        load_slot(1, zo, zo + ldz);
    }
    // Both halves always run (an odd chunk ends with one step whose results are discarded), and
    // the loads of every step are unconditional (plane indices clamped into the padded range), so
    // the slots keep fixed registers around the loop.
    for (int z0 = zb; z0 <= ze; z0 += 2) {
#pragma unroll
        for (int ph = 0; ph < 2; ph++) {
            const int z = z0 + ph;
            const bool real = z <= ze;
            const int cs = ph ^ 1; // slot holding plane z
            const int64_t zo = (int64_t)z * ldz;
            load_slot(ph, (int64_t)min(z + 1, nz + 1) * ldz, (int64_t)min(z + 2, nz + 1) * ldz);
#pragma unroll
            for (int r = 0; r < RY; r++) {
                const double2 c = C[r], ym = r == 0 ? HL[cs][0] : C[r - 1], yp = r == RY - 1 ? HL[cs][1] : C[r + 1];
                const double2 zm = P[r], zp = NL[cs][r];
                const double xm0 = lane_from_left<DPP>(c.y, EL[cs][r]);
                const double xp1 = lane_from_right<DPP>(c.x, ER[cs][r]);
                const double wx = newtonish(MODE) ? WL[cs][r].x : 0.0;
                const double wy = newtonish(MODE) ? WL[cs][r].y : 0.0;
                // NEWTON sweep: exp(w) once per point, shared by the operator and the update
                constexpr bool NS = newtonish(MODE) && KIND == 0;
                const double Ax = NS ? newton_A<MODE>(k, wx) : 0.0, Ay = NS ? newton_A<MODE>(k, wy) : 0.0;
                const double Ex = NS ? newton_E<MODE>(wx) : 0.0, Ey = NS ? newton_E<MODE>(wy) : 0.0;
                const double a0 = NS ? newton_op(div_hh(k, stencil_sum<UN>(k, c.x, c.y, xm0, yp.x, ym.x, zp.x, zm.x)), c.x, Ax, Ex)
                                     : op_value<MODE, UN>(k, c.x, c.y, xm0, yp.x, ym.x, zp.x, zm.x, wx);
                const double a1 = NS ? newton_op(div_hh(k, stencil_sum<UN>(k, c.y, xp1, c.x, yp.y, ym.y, zp.y, zm.y)), c.y, Ay, Ey)
                                     : op_value<MODE, UN>(k, c.y, xp1, c.x, yp.y, ym.y, zp.y, zm.y, wy);
                double r0 = 0.0, r1 = 0.0; // residual of the input iterate
                if (KIND != 2 || ADD) {
                    r0 = FL[cs][r].x - a0;
                    r1 = FL[cs][r].y - a1;
                }
                double o0, o1;
                if (NS) {
                    o0 = newton_update<MODE>(k, c.x, r0, Ax, Ex);
                    o1 = newton_update<MODE>(k, c.y, r1, Ay, Ey);
                } else if (KIND == 0) {
                    o0 = jacobi_update<MODE>(k, c.x, r0, wx);
                    o1 = jacobi_update<MODE>(k, c.y, r1, wy);
                } else if (KIND == 1) {
                    o0 = r0;
                    o1 = r1;
                } else {
                    o0 = ADD ? FL[cs][r].x + a0 : a0;
                    o1 = ADD ? FL[cs][r].y + a1 : a1;
                }
                const bool rowok = real && y0 + r <= ny;
                if (KIND != 2 && partials) {
                    if (rowok && okx0) sumsq += r0 * r0;
                    if (rowok && okx1) sumsq += r1 * r1;
                }
                if (rowok && (KIND != 1 || out)) {
                    double* q = out + x + roff[r + 1] + zo;
                    if (okx1) st2s<NT>(q, o0, o1);
                    else if (okx0) *q = o0;
                }
            }
#pragma unroll
            for (int r = 0; r < RY; r++) {
                P[r] = C[r];
                C[r] = NL[cs][r];
            }
        }
    }
    if (KIND != 2 && partials) {
        const double t = block_sum<W>(sumsq, red);
        if (threadIdx.x == 0 && threadIdx.y == 0) partials[tile] = t;
    }
}

// compF right after findError's update (NewtonSolver.cpp:105-107 then :48-81): w' = w + e (newtonV +=
// v, the expression of k_axpy with a = 1) is formed from both operands wherever the stencil reads it and
// stored once for the block's own points, and the NONLINEAR residual f = F - N(w') with its per-block
// sum of squares is written in the same pass: 40 instead of 48 B per point (k_axpy + k_rb KIND 1).
// Same shape, grid, term order and partial-sum order as k_rb<NONLINEAR, 1> under pass_plan, so f, the
// partials and the norm are bit-identical to the two launches; the caller guarantees that wout's
// non-interior cells already hold what k_axpy would leave there (zeros on a whole level).
// RS: findError's restriction of the new newtonV onto level 1 (NewtonSolver.cpp:88-92, CpuSolver.cpp:211-238) in
// the same pass: a wave's two rows are the fine rows 2Y-1, 2Y of coarse row Y (its upper halo row is 2Y+1), a
// lane's pair the fine columns 2X-1, 2X (2X+1 from the next lane), and coarse plane Z is summed at step 2Z+1 from
// the register window of planes 2Z-1 .. 2Z+1 (never from the slot in flight), in the reference's term order:
// bit-identical to gs_restrict of the stored newtonV, whose 1.1 GB re-read at 512^3 it saves. The chunk of
// planes is even; the last chunk runs one step past the level when nz is even (coarse plane nz / 2).
// (three waves per SIMD, as the plain pass has: <= 168 VGPRs for the restriction's rings)
// BF: the next inner solve's GS_NEWTON_B factor of this level in the same pass — bout = bfac_of(w') at the
// block's own points, from the exp(w') of compF's term (evaluated once): that level's gs_newton_bfac pass is not
// needed (the coarse level's factor stays a gs_newton_bfac pass: its exp inside the restriction's register rings
// spilled ~90 B per lane at three waves per SIMD). RS + BF runs at two waves per SIMD (at three it spills 20 B)
template <int RY, int W, bool UN, bool RS = false, bool BF = false>
__global__ __launch_bounds__(WAVE* W, (RS && BF) ? 2 : 3) void k_newton_upd(Coef k, const double* __restrict__ w,
                                                         const double* __restrict__ e, const double* __restrict__ F,
                                                         double* __restrict__ wout, double* __restrict__ fout,
                                                         double* __restrict__ partials, int nx, int ny, int nz,
                                                         int64_t ldy, int64_t ldz, int ZC, double* __restrict__ cw,
                                                         int cnx, int cny, int cnz, int64_t cldy, int64_t cldz,
                                                         double* __restrict__ bout)
{
    static_assert(!RS || RY == 2, "the restriction takes two fine rows per wave");
    __shared__ double red[W];
    const int lane = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.y);
    const int64_t tile = blockIdx.x + gridDim.x * ((int64_t)blockIdx.y + gridDim.y * (int64_t)blockIdx.z);
    const int x0 = 1 + blockIdx.x * (2 * WAVE);
    const int x = x0 + 2 * lane;
    const int xl = min(x, nx + 1);
    const int y0 = 1 + (blockIdx.y * W + wv) * RY;
    const int zb = 1 + blockIdx.z * ZC;
    const int ze = min(zb + ZC - 1, nz);
    const int zlast = (RS && ze == nz) ? nz + 1 : ze;
    const int xle = x0 - 1;
    const int xre = min(x0 + 2 * WAVE, nx + 1);
    const bool okx0 = x <= nx, okx1 = x + 1 <= nx;
    int64_t roff[RY + 2];
#pragma unroll
    for (int r = 0; r < RY + 2; r++) roff[r] = (int64_t)min(y0 - 1 + r, ny + 1) * ldy;
    auto lw2 = [&](int64_t o) {
        const double2 a = ld2(w + o), b = ld2(e + o);
        return make_double2(a.x + b.x, a.y + b.y);
    };
    auto lw1 = [&](int64_t o) { return w[o] + e[o]; };
    // the ring of k_rb: plane z+1's halo rows, F, edges and plane z+2's rows in slot ph
    double2 P[RY], C[RY], NL[2][RY], FL[2][RY], HL[2][2];
    double EL[2][RY], ER[2][RY];
    // RS: own rows at plane z-2, the upper halo row at planes z-1 / z-2, and the right-edge column (rows 2Y-1,
    // 2Y, 2Y+1) at planes z-1 / z-2; EH: the halo row's right edge in the slot
    double2 PP[RS ? RY : 1], Hh1, Hh2;
    double EH[2], E1[3], E2[3];
    double sumsq = 0.0;
    auto load_slot = [&](const int s, const int64_t z1, const int64_t z2) {
#pragma unroll
        for (int r = 0; r < RY; r++) {
            NL[s][r] = lw2(xl + roff[r + 1] + z2);
            FL[s][r] = ld2s<true>(F + xl + roff[r + 1] + z1);
            EL[s][r] = lw1(xle + roff[r + 1] + z1);
            ER[s][r] = lw1(xre + roff[r + 1] + z1);
        }
        HL[s][0] = lw2(xl + roff[0] + z1);
        HL[s][1] = lw2(xl + roff[RY + 1] + z1);
        if constexpr (RS) EH[s] = lw1(xre + roff[RY + 1] + z1);
    };
    if (zb <= ze) {
        const int64_t zo = (int64_t)zb * ldz;
#pragma unroll
        for (int r = 0; r < RY; r++) {
            P[r] = lw2(xl + roff[r + 1] + zo - ldz);
            C[r] = lw2(xl + roff[r + 1] + zo);
        }
        if constexpr (RS) {
#pragma unroll
            for (int r = 0; r < RY; r++) {
                PP[r] = lw2(xl + roff[r + 1] + zo - 2 * ldz);
                E1[r] = lw1(xre + roff[r + 1] + zo - ldz);
                E2[r] = lw1(xre + roff[r + 1] + zo - 2 * ldz);
            }
            Hh1 = lw2(xl + roff[RY + 1] + zo - ldz);
            Hh2 = lw2(xl + roff[RY + 1] + zo - 2 * ldz);
            E1[2] = lw1(xre + roff[RY + 1] + zo - ldz);
            E2[2] = lw1(xre + roff[RY + 1] + zo - 2 * ldz);
        }
        load_slot(1, zo, zo + ldz);
    }
    const int X = 1 + (int)blockIdx.x * WAVE + lane, Yc = (y0 + 1) / 2;
    for (int z0 = zb; z0 <= zlast; z0 += 2) {
#pragma unroll
        for (int ph = 0; ph < 2; ph++) {
            const int z = z0 + ph;
            const bool real = z <= ze;
            const int cs = ph ^ 1;
            const int64_t zo = (int64_t)z * ldz;
            load_slot(ph, (int64_t)min(z + 1, nz + 1) * ldz, (int64_t)min(z + 2, nz + 1) * ldz);
#pragma unroll
            for (int r = 0; r < RY; r++) {
                const double2 c = C[r], ym = r == 0 ? HL[cs][0] : C[r - 1], yp = r == RY - 1 ? HL[cs][1] : C[r + 1];
                const double2 zm = P[r], zp = NL[cs][r];
                const double xm0 = lane_from_left<true>(c.y, EL[cs][r]);
                const double xp1 = lane_from_right<true>(c.x, ER[cs][r]);
                // (compF's non-linear term gamma w' exp(w'), NewtonSolver.cpp:63-72, and B share exp(w'))
                double a0 = div_hh(k, stencil_sum<UN>(k, c.x, c.y, xm0, yp.x, ym.x, zp.x, zm.x));
                double a1 = div_hh(k, stencil_sum<UN>(k, c.y, xp1, c.x, yp.y, ym.y, zp.y, zm.y));
                double b0 = 0.0, b1 = 0.0;
                {
                    const double E0 = exp(c.x), E1 = exp(c.y);
                    const double nl0 = k.gamma * c.x * E0, nl1 = k.gamma * c.y * E1;
                    a0 += nl0;
                    a1 += nl1;
                    if constexpr (BF) {
                        b0 = k.gamma * (1 + c.x) * E0;
                        b1 = k.gamma * (1 + c.y) * E1;
                    }
                }
                const double r0 = FL[cs][r].x - a0, r1 = FL[cs][r].y - a1;
                const bool rowok = real && y0 + r <= ny;
                if (rowok && okx0) sumsq += r0 * r0;
                if (rowok && okx1) sumsq += r1 * r1;
                if (rowok) {
                    const int64_t q = x + roff[r + 1] + zo;
                    if (okx1) {
                        st2s<true>(fout + q, r0, r1);
                        st2s<true>(wout + q, c.x, c.y);
                        if constexpr (BF) st2s<true>(bout + q, b0, b1);
                    } else if (okx0) {
                        fout[q] = r0;
                        wout[q] = c.x;
                        if constexpr (BF) bout[q] = b0;
                    }
                }
            }
            if constexpr (RS) {
                // coarse plane Z = (z - 1) / 2 from planes z-2 (PP), z-1 (P), z (C): fine (2X+ii, 2Y+jj, 2Z+kk)
                const int Zc = (z - 1) >> 1;
                const bool odd = z & 1;
                // the fine column 2X+1 of each (row, plane): the next lane's 2X-1, the edge column for lane 63
                const double2 rows[3][3] = {{PP[0], PP[1], Hh2}, {P[0], P[1], Hh1}, {C[0], C[1], HL[cs][1]}};
                const double eg[3][3] = {{E2[0], E2[1], E2[2]}, {E1[0], E1[1], E1[2]}, {ER[cs][0], ER[cs][1], EH[cs]}};
                if (odd && Zc >= 1 && Zc <= cnz) { // (wave-uniform; the DPP shifts need every lane)
                    double acc = 0.0;
#pragma unroll
                    for (int ii = -1; ii <= 1; ii++)
#pragma unroll
                        for (int jj = -1; jj <= 1; jj++)
#pragma unroll
                            for (int kk = -1; kk <= 1; kk++) {
                                const double fac = 0.125 * ((2.0 - (ii < 0 ? -ii : ii)) / 2.0) *
                                                   ((2.0 - (jj < 0 ? -jj : jj)) / 2.0) *
                                                   ((2.0 - (kk < 0 ? -kk : kk)) / 2.0);
                                const double2 v2 = rows[kk + 1][jj + 1];
                                const double t = ii < 0 ? v2.x
                                                        : (ii == 0 ? v2.y
                                                                   : lane_from_right<true>(v2.x, eg[kk + 1][jj + 1]));
                                acc += fac * t;
                            }
                    if (X <= cnx && Yc <= cny) cw[X + (int64_t)Yc * cldy + (int64_t)Zc * cldz] = acc;
                }
                Hh2 = Hh1;
                Hh1 = HL[cs][1];
#pragma unroll
                for (int i = 0; i < 3; i++) E2[i] = E1[i];
                E1[0] = ER[cs][0];
                E1[1] = ER[cs][1];
                E1[2] = EH[cs];
#pragma unroll
                for (int r = 0; r < RY; r++) PP[r] = P[r];
            }
#pragma unroll
            for (int r = 0; r < RY; r++) {
                P[r] = C[r];
                C[r] = NL[cs][r];
            }
        }
    }
    if (partials) {
        const double t = block_sum<W>(sumsq, red);
        if (threadIdx.x == 0 && threadIdx.y == 0) partials[tile] = t;
    }
}

dim3 rb_grid(const gs_level* L, int RY, int W, int ZC, bool oneD = false)
{
    const dim3 g((unsigned)((L->nx + 2 * WAVE - 1) / (2 * WAVE)), (unsigned)((L->ny + RY * W - 1) / (RY * W)),
                 (unsigned)((L->nz + ZC - 1) / ZC));
    return oneD ? dim3(g.x * g.y * g.z) : g;
}

// ---------------------------------------------------------------------------------------------
// Generic-stencil pass (any 7 offsets in {-1,0,1}^3, any order): one point per thread.
constexpr int GN_BX = 64, GN_BY = 4;

template <int MODE, int KIND, bool ADD>
__global__ __launch_bounds__(256) void k_generic(Coef k, const double* __restrict__ v, const double* __restrict__ f,
                                                 const double* __restrict__ w, double* __restrict__ out,
                                                 double* __restrict__ partials, int nx, int ny, int nz, int64_t ldy,
                                                 int64_t ldz)
{
    __shared__ double red[GN_BY];
    const int x = 1 + blockIdx.x * GN_BX + threadIdx.x;
    const int y = 1 + blockIdx.y * GN_BY + threadIdx.y;
    const int z = 1 + blockIdx.z;
    double sumsq = 0.0;
    if (x <= nx && y <= ny) {
        const int64_t p = x + y * ldy + (int64_t)z * ldz;
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 7; i++) s += k.s[i] * (v ? v[p + k.off[i]] : 0.0);
        s = div_hh(k, s);
        const double c = v ? v[p] : 0.0;
        const double wv = newtonish(MODE) ? w[p] : 0.0;
        s = op_finish<MODE>(k, s, c, wv);
        if (KIND == 0) {
            const double r = f[p] - s;
            sumsq = r * r;
            out[p] = jacobi_update<MODE>(k, c, r, wv);
        } else if (KIND == 1) {
            const double r = f[p] - s;
            sumsq = r * r;
            if (out) out[p] = r;
        } else {
            out[p] = ADD ? out[p] + s : s;
        }
    }
    if (KIND != 2 && partials) {
        const double t = block_sum<GN_BY>(sumsq, red);
        if (threadIdx.x == 0 && threadIdx.y == 0)
            partials[blockIdx.x + gridDim.x * ((int64_t)blockIdx.y + gridDim.y * (int64_t)blockIdx.z)] = t;
    }
}

dim3 gn_grid(const gs_level* L)
{
    return dim3((unsigned)((L->nx + GN_BX - 1) / GN_BX), (unsigned)((L->ny + GN_BY - 1) / GN_BY), (unsigned)L->nz);
}

// ---------------------------------------------------------------------------------------------
// Deterministic finish of the per-block partial sums: one block, fixed strided order.
constexpr int FIN_T = 1024;
__global__ __launch_bounds__(FIN_T) void k_sumsq_finish(const double* __restrict__ partials, int64_t n,
                                                        double* __restrict__ out, int accumulate)
{
    __shared__ double red[FIN_T / WAVE];
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += FIN_T) s += partials[i];
    const double t = block_sum<FIN_T / WAVE>(s, red);
    if (threadIdx.x == 0) *out = accumulate ? t : sqrt(t);
}

// ---------------------------------------------------------------------------------------------
// 27-point full weighting (CpuSolver.cpp:211-238): coarse interior point per thread, terms summed
// with ii outermost, kk innermost. The weights are exact powers of two.
// Z-slabs: coarse local plane z is global z + cz0, its centre fine plane global 2(z + cz0), local
// 2(z + cz0) - fz0 (both z0 = 0 on an unpartitioned level).
__global__ __launch_bounds__(256) void k_restrict(const double* __restrict__ fine, double* __restrict__ ca,
                                                  double* __restrict__ cb, int cnx, int cny, int cnz, int64_t fldy,
                                                  int64_t fldz, int64_t cldy, int64_t cldz, int zoff)
{
    const int x = 1 + blockIdx.x * 64 + threadIdx.x;
    const int y = 1 + blockIdx.y * 4 + threadIdx.y;
    const int z = 1 + blockIdx.z;
    if (x > cnx || y > cny) return;
    const double* c0 = fine + 2 * x + (int64_t)(2 * y) * fldy + (int64_t)(2 * z + zoff) * fldz;
    double acc = 0.0;
#pragma unroll
    for (int a = -1; a <= 1; a++)
#pragma unroll
        for (int b = -1; b <= 1; b++)
#pragma unroll
            for (int c = -1; c <= 1; c++) {
                const double wgt = 0.125 * ((2.0 - (a < 0 ? -a : a)) / 2.0) * ((2.0 - (b < 0 ? -b : b)) / 2.0) *
                                   ((2.0 - (c < 0 ? -c : c)) / 2.0);
                acc += wgt * c0[a + b * fldy + c * fldz];
            }
    const int64_t q = x + y * cldy + (int64_t)z * cldz;
    ca[q] = acc;
    if (cb) cb[q] = acc;
}

// ---------------------------------------------------------------------------------------------
// Residual fused into the full-weighting restriction: coarse f = R(f - A v) without writing the fine
// residual to memory (CpuSolver.cpp:45-83 then :211-238; the reference stores r and re-reads it).
// A block owns RR_TXC x RR_TYC coarse columns and marches a chunk of coarse planes. The fine region
// its 27-point stencils touch is (2 RR_TXC + 1) x (2 RR_TYC + 1) points per plane; the v tile with its
// one-point halo is staged in a 4-plane LDS ring (loaded once, coalesced along x), the residual of
// that region in a 3-plane LDS ring. Per coarse plane Z: the two new v planes and the f values of the
// next plane pair are loaded into registers while the current ones are computed (software pipeline),
// r is evaluated on fine planes 2Z and 2Z+1 (2Z-1 is kept from the previous plane), then every
// thread sums its coarse point's 27 terms in the reference's order. Fine points outside the interior
// hold r = 0, as the reference's never-written boundary does. Each residual is the gs_residual
// expression and each sum the gs_restrict one: bit-identical to the unfused pair.
constexpr int RR_TXC = 64, RR_TYC = 4, RR_T = RR_TXC * RR_TYC;
constexpr int RR_FX = 2 * RR_TXC + 1, RR_FY = 2 * RR_TYC + 1; // residual region per plane
constexpr int RR_VX = RR_FX + 2, RR_VY = RR_FY + 2;           // v tile per plane (one-point halo)
constexpr int RR_NR = (RR_FX * RR_FY + RR_T - 1) / RR_T;      // residual points per thread and plane
constexpr int RR_NV = (RR_VX * RR_VY + RR_T - 1) / RR_T;      // v tile points per thread and plane

struct StencilOffsets {
    int lds[7]; // ox + oy * RR_VX (in-plane LDS offset)
    int oz[7];
};

template <int MODE>
__global__ __launch_bounds__(RR_T) void k_resrestrict(Coef k, StencilOffsets so, const double* __restrict__ v,
                                                      const double* __restrict__ f, const double* __restrict__ w,
                                                      double* __restrict__ ca, double* __restrict__ cb, int fnx,
                                                      int fny, int fnz, int64_t fldy, int64_t fldz, int cnx, int cny,
                                                      int cnz, int64_t cldy, int64_t cldz, int zoff, int ZC)
{
    // one LDS array addressed with integer offsets (pointers into it would become flat accesses):
    // v ring slots 0..3 at s * RR_VP, residual ring slots 0..2 at 4 RR_VP + s * RR_RP
    constexpr int RR_VP = RR_VY * RR_VX, RR_RP = RR_FY * RR_FX;
    __shared__ double lds[4 * RR_VP + 3 * RR_RP];
    const int tid = threadIdx.x;
    // (an XCD-aware tile order, as k_tb2y uses, measured 3% slower here: tools/ab_session.sh)
    const int X0 = 1 + blockIdx.x * RR_TXC, Y0 = 1 + blockIdx.y * RR_TYC;
    const int Zb = 1 + blockIdx.z * ZC, Ze = min(Zb + ZC - 1, cnz);
    if (Zb > Ze) return;
    const int fx0 = 2 * X0 - 1, fy0 = 2 * Y0 - 1; // residual region origin (fine)

    // this thread's v-tile points (clamped into the padded level: clamped copies are never used)
    int64_t voff[RR_NV];
#pragma unroll
    for (int i = 0; i < RR_NV; i++) {
        const int e = min(tid + i * RR_T, RR_VX * RR_VY - 1);
        const int ly = e / RR_VX, lx = e - ly * RR_VX;
        voff[i] = min(fx0 - 1 + lx, fnx + 1) + (int64_t)min(fy0 - 1 + ly, fny + 1) * fldy;
    }
    // this thread's residual points: global offset, LDS position, interior flag
    int64_t roff[RR_NR];
    int rpos[RR_NR];
    bool rin[RR_NR];
#pragma unroll
    for (int i = 0; i < RR_NR; i++) {
        const int e = tid + i * RR_T;
        const int ry = min(e, RR_FX * RR_FY - 1) / RR_FX, rx = min(e, RR_FX * RR_FY - 1) - ry * RR_FX;
        const int x = fx0 + rx, y = fy0 + ry;
        rin[i] = e < RR_FX * RR_FY && x <= fnx && y <= fny;
        roff[i] = min(x, fnx + 1) + (int64_t)min(y, fny + 1) * fldy;
        rpos[i] = (ry + 1) * RR_VX + rx + 1;
    }
    auto zc = [&](int fz) { return (int64_t)min(max(fz, -1), fnz + 2) * fldz; };
    auto load_v = [&](double (&dst)[RR_NV], int fz) {
        const int64_t zo = zc(fz);
#pragma unroll
        for (int i = 0; i < RR_NV; i++) dst[i] = v[voff[i] + zo];
    };
    auto store_v = [&](const double (&src)[RR_NV], int fz) {
        const int d = ((fz + 4) & 3) * RR_VP;
#pragma unroll
        for (int i = 0; i < RR_NV; i++)
            if (tid + i * RR_T < RR_VP) lds[d + tid + i * RR_T] = src[i];
    };
    auto load_fw = [&](double (&F)[RR_NR], double (&W)[RR_NR], int fz) {
        const int64_t zo = zc(fz);
#pragma unroll
        for (int i = 0; i < RR_NR; i++) {
            F[i] = f[roff[i] + zo];
            if (newtonish(MODE)) W[i] = w[roff[i] + zo];
        }
    };
    // r on fine plane fz from the v ring (needs planes fz-1 .. fz+1 staged)
    auto residual_plane = [&](const double (&F)[RR_NR], const double (&W)[RR_NR], int fz) {
        int toff[7]; // LDS offset of each stencil term relative to the point's in-plane position
#pragma unroll
        for (int t = 0; t < 7; t++) toff[t] = ((fz + 4 + so.oz[t]) & 3) * RR_VP + so.lds[t];
        const int coff = ((fz + 4) & 3) * RR_VP;
        const int dst = 4 * RR_VP + ((fz + 3) % 3) * RR_RP;
        const bool zin = fz >= 1 && fz <= fnz;
#pragma unroll
        for (int i = 0; i < RR_NR; i++) {
            if (tid + i * RR_T >= RR_FX * RR_FY) continue;
            double r = 0.0;
            if (zin && rin[i]) {
                double sum = 0.0;
#pragma unroll
                for (int t = 0; t < 7; t++) sum += k.s[t] * lds[rpos[i] + toff[t]];
                const double c = lds[rpos[i] + coff];
                const double q = op_finish<MODE>(k, div_hh(k, sum), c, newtonish(MODE) ? W[i] : 0.0);
                r = F[i] - q;
            }
            lds[dst + tid + i * RR_T] = r;
        }
    };

    double VA[RR_NV], VB[RR_NV], FA[RR_NR], FB[RR_NR], WA[RR_NR], WB[RR_NR];
    // prologue: v planes P-2 .. P (P = 2 Zb + zoff) into the ring, r(P-1)
    const int P0 = 2 * Zb + zoff;
    load_v(VA, P0 - 2);
    load_v(VB, P0 - 1);
    load_fw(FA, WA, P0 - 1);
    store_v(VA, P0 - 2);
    store_v(VB, P0 - 1);
    load_v(VA, P0);
    store_v(VA, P0);
    __syncthreads();
    residual_plane(FA, WA, P0 - 1);
    // staged for the first step: v(P+1), v(P+2), f(P), f(P+1)
    load_v(VA, P0 + 1);
    load_v(VB, P0 + 2);
    load_fw(FA, WA, P0);
    load_fw(FB, WB, P0 + 1);
    __syncthreads(); // v(P+2) goes to the slot of v(P-2), which r(P-1) just read
    const int cx = tid % RR_TXC, cy = tid / RR_TXC;
    const int X = X0 + cx, Y = Y0 + cy;
    for (int Z = Zb; Z <= Ze; Z++) {
        const int P = 2 * Z + zoff;
        store_v(VA, P + 1);
        store_v(VB, P + 2);
        __syncthreads();
        double F0[RR_NR], F1[RR_NR], W0[RR_NR], W1[RR_NR];
#pragma unroll
        for (int i = 0; i < RR_NR; i++) {
            F0[i] = FA[i];
            F1[i] = FB[i];
            W0[i] = WA[i];
            W1[i] = WB[i];
        }
        if (Z < Ze) { // the next step's operands, in flight during this step's arithmetic
            load_v(VA, P + 3);
            load_v(VB, P + 4);
            load_fw(FA, WA, P + 2);
            load_fw(FB, WB, P + 3);
        }
        residual_plane(F0, W0, P);
        residual_plane(F1, W1, P + 1);
        __syncthreads();
        if (X <= cnx && Y <= cny) {
            double acc = 0.0;
#pragma unroll
            for (int a = -1; a <= 1; a++)
#pragma unroll
                for (int b = -1; b <= 1; b++)
#pragma unroll
                    for (int c = -1; c <= 1; c++) {
                        const double wgt = 0.125 * ((2.0 - (a < 0 ? -a : a)) / 2.0) * ((2.0 - (b < 0 ? -b : b)) / 2.0) *
                                           ((2.0 - (c < 0 ? -c : c)) / 2.0);
                        acc += wgt * lds[4 * RR_VP + ((P + c + 3) % 3) * RR_RP + (2 * cy + 1 + b) * RR_FX + 2 * cx + 1 + a];
                    }
            const int64_t q = X + Y * cldy + (int64_t)Z * cldz;
            ca[q] = acc;
            if (cb) cb[q] = acc;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Residual + full weighting in registers ("rr2": canonical stencil order, all three modes, levels
// or Z-slabs (zhi) of rows <= 1024 points). A block is the whole row of coarse columns of ONE
// coarse row Y (WX waves of 64 lanes; lane = coarse column X, its fine pair x = 2X-1, 2X one dwordx4)
// and marches a chunk of coarse planes. Per coarse plane Z it evaluates the residual on fine planes 2Z
// and 2Z+1 (2Z-1 is kept from the previous plane) for the three fine rows 2Y-1 .. 2Y+1 the 27-point sum
// reads (row 2Y+1 is also the next row's first: recomputed there, its loads hit L2) the way k_rb's
// residual pass does: x-neighbours by DPP lane shifts with the wave-edge columns exchanged through LDS
// (zero beyond the level's x-boundaries, which hold v = 0), y-neighbours from the lane's own rows plus
// two halo rows, z-neighbours from the register window. r at the next coarse column's first fine
// column (2X+1) is one more DPP shift (the right wave's lane 0 through LDS). The 27 terms are summed in
// the reference's order (CpuSolver.cpp:225-231): 16 B of compulsory HBM reads per fine point (v, f)
// plus 1 B of coarse writes, the residual never stored, and no LDS staging of the operands (the
// LDS-tiled k_resrestrict, kept for the other cases, is latency-bound at 2 blocks per CU). PF = true
// keeps the next coarse plane's loads in flight (two-slot ring, as in k_rb); production runs PF =
// false: one slot loaded per step, 154 VGPRs and 3 waves per SIMD, measured faster. Blocks go in
// XCD-aware order, y fastest, so the neighbouring rows that share 3 of a block's 5 v rows run on the
// same XCD at the same time.
constexpr int RR2_WXMAX = 8, RR2_NR2_LOG2_POINTS = 26;

// NR: coarse rows per block (1: fine rows 2Y-1..2Y+1 computed; 2: 2Y-1..2Y+3, the shared row 2Y+1 and three
// of the seven v rows once instead of twice)
// NG: groups of WX waves per block, group g owning coarse rows Y + NR g: the groups are y-neighbours that march
// the same planes in lock-step (the per-plane barrier is the block's), so the v / f rows they share are
// fetched by the one CU at the same time — an L1 / L2 hit for the second group — instead of by two blocks
// that drift apart on different CUs (where the shared rows miss the 4 MB L2 a third of the time)
template <int MODE, bool PF, int NR = 1, bool UN = false, bool NTU = false, int NG = 1> // PF: the next plane's operands in flight (two-slot ring), else loaded per step
__global__ __launch_bounds__(WAVE* RR2_WXMAX) void k_rr2(Coef k, const double* __restrict__ v,
                                                         const double* __restrict__ f, const double* __restrict__ w,
                                                         double* __restrict__ ca,
                                                         double* __restrict__ cb, int fnx, int fny, int fnz,
                                                         int64_t fldy, int64_t fldz, int cnx, int cny, int cnz, int64_t cldy,
                                                         int64_t cldz, int ZC, int zhi, int rev)
{
    static_assert(!newtonish(MODE) || !PF, "NEWTON: newtonV rows exceed the budget of the prefetch ring");
    constexpr int RR = 2 * NR + 1; // computed fine rows; v rows 0 .. RR+1 (0 and RR+1: halo rows)
    // wave-edge columns [parity][1 + wave][side][plane * 3 + row] of v, and r at each wave's first fine
    // column [parity][1 + wave][plane * 3 + row]; slots 0 and WX+1 are the zero x-boundary
    __shared__ double veA[NG][2][RR2_WXMAX + 2][2][2 * RR];
    __shared__ double reA[NG][2][RR2_WXMAX + 2][2 * RR];
    const int lane = threadIdx.x;
    const int wx = __builtin_amdgcn_readfirstlane(threadIdx.y);
    const int grp = NG > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.z) : 0;
    const int WX = blockDim.y;
    const int tid = lane + WAVE * (wx + WX * grp);
    for (int i = tid; i < NG * 2 * (RR2_WXMAX + 2) * 2 * 2 * RR; i += WAVE * WX * NG) (&veA[0][0][0][0][0])[i] = 0.0;
    for (int i = tid; i < NG * 2 * (RR2_WXMAX + 2) * 2 * RR; i += WAVE * WX * NG) (&reA[0][0][0][0])[i] = 0.0;
    __syncthreads();
    double (&ve)[2][RR2_WXMAX + 2][2][2 * RR] = veA[grp]; // this group's wave-edge exchange
    double (&re)[2][RR2_WXMAX + 2][2 * RR] = reA[grp];
    const int64_t tile = xcd_tile(blockIdx.x + (int64_t)gridDim.x * blockIdx.y, (int64_t)gridDim.x * gridDim.y);
    const int Y = 1 + NR * (NG * (int)(tile % gridDim.x) + grp);
    // rev (GS_RR_REVERSE): the z-chunks in descending order, so the first blocks read the planes the
    // preceding pair launch touched last
    const int zi = (int)(tile / gridDim.x);
    const int Zb = 1 + (rev ? (int)gridDim.y - 1 - zi : zi) * ZC, Ze = min(Zb + ZC - 1, cnz);
    const int X = 1 + wx * WAVE + lane;
    const int x = 2 * X - 1, xl = min(x, fnx + 1);
    const bool okx0 = x <= fnx, okx1 = x + 1 <= fnx;
    int64_t roff[RR + 2]; // fine rows 2Y-2 .. 2Y+2NR (computed: 1..RR)
    bool rowc[RR + 2];
#pragma unroll
    for (int j = 0; j < RR + 2; j++) {
        const int y = 2 * Y - 2 + j;
        roff[j] = (int64_t)min(max(y, 0), fny + 1) * fldy;
        rowc[j] = y >= 1 && y <= fny;
    }
    // zhi: plane fnz+1 is an internal Z-slab boundary (current ghost planes fnz+1 of v, f, w and
    // fnz+2 of v): the residual there is real, not the zero of a level boundary
    auto at = [&](const double* b, int j, int p) {
        return b + xl + roff[j] + (int64_t)min(max(p, 0), fnz + 1 + zhi) * fldz;
    };
    // one step's operands: v planes 2Z+1 (A), 2Z+2 (B) of rows 1..3; halo rows 0 / 4 of planes 2Z (H0)
    // and 2Z+1 (H1); f of planes 2Z (F0), 2Z+1 (F1) rows 1..3
    double2 VA[2][RR], VB[2][RR], H0[2][2], H1[2][2], F0[2][RR], F1[2][RR], W0[2][RR], W1[2][RR];
    auto load_slot = [&](const int s, const int Z) {
        const int p = 2 * Z;
        // the step's halo rows first (the rows the y-neighbour blocks read too), then row by row: k_rr2 0.442-0.443 vs
        // 0.458-0.459 ms LINEAR, 0.7085-0.7088 vs 0.7254-0.7259 ms NEWTON_B per 512^3 launch (r06x / r06y,
        // interleaved, profiles/r06/r06x_load_order_ab.txt; f rows first: 0.449 / 0.726-0.740, plane by plane: 0.484-0.485 /
        // 0.754-0.760, v / f / w grouped: 0.481-0.485 / 0.747-0.750, halos then v then f / w: 0.476-0.478 / 0.751)
        H0[s][0] = ld2(at(v, 0, p));
        H0[s][1] = ld2(at(v, RR + 1, p));
        H1[s][0] = ld2(at(v, 0, p + 1));
        H1[s][1] = ld2(at(v, RR + 1, p + 1));
#pragma unroll
        for (int j = 0; j < RR; j++) {
            // NTU: rows no neighbouring block reads (v: 2Y+1 .. 2Y+2NR-3, f: 2Y .. 2Y+2NR-2) bypass L2
            // retention, leaving it to the shared halo rows
            const bool uv = NTU && j >= 2 && j <= RR - 3, uf = NTU && j >= 1 && j <= RR - 2;
            VA[s][j] = uv ? ld2s<true>(at(v, j + 1, p + 1)) : ld2(at(v, j + 1, p + 1));
            VB[s][j] = uv ? ld2s<true>(at(v, j + 1, p + 2)) : ld2(at(v, j + 1, p + 2));
            F0[s][j] = uf ? ld2s<true>(at(f, j + 1, p)) : ld2(at(f, j + 1, p));
            F1[s][j] = uf ? ld2s<true>(at(f, j + 1, p + 1)) : ld2(at(f, j + 1, p + 1));
            if (MODE == GS_NEWTON_B && k.bconst) {
                W0[s][j] = make_double2(k.gamma, k.gamma);
                W1[s][j] = W0[s][j];
            } else if (newtonish(MODE)) {
                W0[s][j] = uf ? ld2s<true>(at(w, j + 1, p)) : ld2(at(w, j + 1, p));
                W1[s][j] = uf ? ld2s<true>(at(w, j + 1, p + 1)) : ld2(at(w, j + 1, p + 1));
            }
        }
    };
    // LDS-only barrier: the outstanding prefetch stays in flight across it
    auto lds_barrier = [] { GS_LDS_BARRIER(); }; // lgkmcnt(0), s_barrier
    // the columns left of lane 0 / right of lane 63 on two planes: v(x-1) of lane 0, v(x+2) of lane 63
    auto edges_v = [&](int par, const double2 (&P)[RR], const double2 (&Q)[RR], double (&CLp)[RR], double (&CRp)[RR],
                       double (&CLq)[RR], double (&CRq)[RR]) {
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < RR; j++) {
                ve[par][wx + 1][0][j] = P[j].x;
                ve[par][wx + 1][0][RR + j] = Q[j].x;
            }
        }
        if (lane == WAVE - 1) {
#pragma unroll
            for (int j = 0; j < RR; j++) {
                ve[par][wx + 1][1][j] = P[j].y;
                ve[par][wx + 1][1][RR + j] = Q[j].y;
            }
        }
        lds_barrier();
#pragma unroll
        for (int j = 0; j < RR; j++) {
            CLp[j] = uniform_d(ve[par][wx][1][j]);
            CRp[j] = uniform_d(ve[par][wx + 2][0][j]);
            CLq[j] = uniform_d(ve[par][wx][1][RR + j]);
            CRq[j] = uniform_d(ve[par][wx + 2][0][RR + j]);
        }
    };
    // r(2X+1) of every lane for two planes: the right neighbour lane's r.x (lane 63: the right wave's)
    auto edges_r = [&](int par, const double2 (&R)[RR], const double2 (&S)[RR], double (&NQ)[RR], double (&NS)[RR]) {
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < RR; j++) {
                re[par][wx + 1][j] = R[j].x;
                re[par][wx + 1][RR + j] = S[j].x;
            }
        }
        lds_barrier();
#pragma unroll
        for (int j = 0; j < RR; j++) {
            NQ[j] = lane_from_right<true>(R[j].x, uniform_d(re[par][wx + 2][j]));
            NS[j] = lane_from_right<true>(S[j].x, uniform_d(re[par][wx + 2][RR + j]));
        }
    };
    // r = f - A v on fine plane p, rows 1..3 (k_rb KIND 1: same expression, same term order); 0 outside
    // the interior, as the reference's never-written boundary of r
    auto resid = [&](const double2 (&Vm)[RR], const double2 (&Vc)[RR], const double2 (&H)[2], const double2 (&Vp)[RR],
                     const double2 (&F)[RR], const double2 (&W)[RR], const double (&CL)[RR], const double (&CR)[RR], int p,
                     double2 (&R)[RR]) {
        const bool pin = p >= 1 && (p <= fnz || (zhi && p == fnz + 1));
#pragma unroll
        for (int j = 0; j < RR; j++) {
            const double2 c = Vc[j];
            const double2 ym = j == 0 ? H[0] : Vc[j - 1], yp = j == RR - 1 ? H[1] : Vc[j + 1];
            const double xm0 = lane_from_left<true>(c.y, CL[j]);
            const double xp1 = lane_from_right<true>(c.x, CR[j]);
            const double w0 = newtonish(MODE) ? W[j].x : 0.0, w1 = newtonish(MODE) ? W[j].y : 0.0;
            const double a0 = op_value<MODE, UN>(k, c.x, c.y, xm0, yp.x, ym.x, Vp[j].x, Vm[j].x, w0);
            const double a1 = op_value<MODE, UN>(k, c.y, xp1, c.x, yp.y, ym.y, Vp[j].y, Vm[j].y, w1);
            const bool ok = pin && rowc[j + 1];
            R[j] = make_double2((ok && okx0) ? F[j].x - a0 : 0.0, (ok && okx1) ? F[j].y - a1 : 0.0);
        }
    };

    // prologue: r on fine plane 2Zb-1 (the top plane of the previous coarse plane's stencil)
    double2 Vm[RR], V0[RR], Rm[RR];
    double Nm[RR];
    {
        const int p = 2 * Zb - 1;
        double2 Vq[RR], Hq[2], Fq[RR], Wq[RR];
#pragma unroll
        for (int j = 0; j < RR; j++) {
            Vm[j] = ld2(at(v, j + 1, p - 1));
            Vq[j] = ld2(at(v, j + 1, p));
            V0[j] = ld2(at(v, j + 1, p + 1));
            Fq[j] = ld2(at(f, j + 1, p));
            Wq[j] = (MODE == GS_NEWTON_B && k.bconst) ? make_double2(k.gamma, k.gamma)
                    : newtonish(MODE)                  ? ld2(at(w, j + 1, p))
                                                       : make_double2(0.0, 0.0);
        }
        Hq[0] = ld2(at(v, 0, p));
        Hq[1] = ld2(at(v, RR + 1, p));
        double CL[RR], CR[RR], CL2[RR], CR2[RR], N2[RR];
        edges_v(1, Vq, Vq, CL, CR, CL2, CR2);
        resid(Vm, Vq, Hq, V0, Fq, Wq, CL, CR, p, Rm);
        edges_r(1, Rm, Rm, Nm, N2);
#pragma unroll
        for (int j = 0; j < RR; j++) Vm[j] = Vq[j]; // window: Vm = v(2Zb-1), V0 = v(2Zb)
    }
    if (PF) load_slot(1, Zb);
    // Both halves always run (an odd chunk ends with a step whose results are discarded), and every
    // load is unconditional (plane indices clamped), so the slots keep fixed registers.
    for (int z0 = Zb; z0 <= Ze; z0 += 2) {
#pragma unroll
        for (int ph = 0; ph < 2; ph++) {
            const int Z = z0 + ph;
            const int cs = PF ? ph ^ 1 : 0; // slot holding this step's operands
            if (PF) load_slot(ph, Z + 1);
            else load_slot(0, Z);
            double CL0[RR], CR0[RR], CL1[RR], CR1[RR];
            edges_v(ph, V0, VA[cs], CL0, CR0, CL1, CR1);
            double2 R0[RR], R1[RR];
            resid(Vm, V0, H0[cs], VA[cs], F0[cs], W0[cs], CL0, CR0, 2 * Z, R0);
            resid(V0, VA[cs], H1[cs], VB[cs], F1[cs], W1[cs], CL1, CR1, 2 * Z + 1, R1);
            double N0[RR], N1[RR];
            edges_r(ph, R0, R1, N0, N1);
#pragma unroll
            for (int i = 0; i < NR; i++) {
                if (Z <= Ze && X <= cnx && Y + i <= cny) {
                    double acc = 0.0;
#pragma unroll
                    for (int a = -1; a <= 1; a++)
#pragma unroll
                        for (int b = -1; b <= 1; b++)
#pragma unroll
                            for (int c = -1; c <= 1; c++) {
                                const double wgt = 0.125 * ((2.0 - (a < 0 ? -a : a)) / 2.0) *
                                                   ((2.0 - (b < 0 ? -b : b)) / 2.0) *
                                                   ((2.0 - (c < 0 ? -c : c)) / 2.0);
                                const int j = 2 * i + b + 1;
                                const double2 rp = c < 0 ? Rm[j] : (c == 0 ? R0[j] : R1[j]);
                                const double rn = c < 0 ? Nm[j] : (c == 0 ? N0[j] : N1[j]);
                                acc += wgt * (a < 0 ? rp.x : (a == 0 ? rp.y : rn));
                            }
                    const int64_t q = X + (Y + i) * cldy + (int64_t)Z * cldz;
                    ca[q] = acc;
                    if (cb) cb[q] = acc;
                }
            }
#pragma unroll
            for (int j = 0; j < RR; j++) {
                Vm[j] = VA[cs][j];
                V0[j] = VB[cs][j];
                Rm[j] = R1[j];
                Nm[j] = N1[j];
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Residual + full weighting with an LDS-DMA operand ring ("rr2d", r06; verdict r05 item 1). Same arithmetic,
// term order and outputs as k_rr2 (bit-identical), built for the case k_rr2 handles worst: its operands of a plane
// step are loaded at the top of the step and waited for at once (no register room for a prefetch ring: PF = false),
// so at two waves per SIMD the loads are exposed every step (PMC wait_inst 0.43-0.46 of wave cycles).
// Here the operands never occupy VGPRs while in flight: every wave streams ITS OWN columns of the operand rows of
// fine plane p + 2 straight into an LDS ring (global_load_lds_dwordx4, one instruction per row and wave, inline asm:
// M0 is written in the statement that reads it) while it computes plane p, and waits for plane p's with a hand-
// counted s_waitcnt vmcnt before the step's one barrier. A ring slot holds what the residual of fine plane p adds to
// the register window (v of planes p-1, p): v of plane p+1 on the computed rows, the two halo rows of plane p, f
// (and NEWTON's w) of plane p, RR + 2 + RR (+ RR) rows of the block's width; three slots (plane p read, p+1 and p+2
// in flight). The wave-edge columns x-1 / x+2 of every v row are read straight from the neighbouring waves' columns
// of the slot (LDS broadcast reads, one plane early), so only r's wave-edge column still goes through an exchange.
// One fine plane per step; the restriction of coarse plane Z runs at step 2Z+2, once r of plane 2Z+1 has crossed
// the wave edges with that step's barrier.
// The counted wait is exact because every VMEM operation of the loop is accounted for: RROWS DMA instructions per
// step and 2 NR coarse stores at every even step, stores that never branch away (an invalid point writes to a sink
// word instead); so before the wait of step p exactly one plane's DMA group and one store group are younger than
// plane p's DMA group (the prologue issues one group of sink stores to make step p0 look the same).
// LDS: 3 slots x RROWS rows x WX KB (512-point rows: 144 KB LINEAR NR = 2, 132 KB NEWTON NR = 1): one block per CU.
constexpr int RR2D_WXMAX = 4, RR2D_SLOTS = 3;
__device__ double gs_rr2d_sink[2 * WAVE]; // where the unconditional stores of invalid points go

template <int MODE, int NR, bool WR>
constexpr int rr2d_rows()
{
    return (2 * NR + 1) * (WR ? 3 : 2) + 2;
}

template <int N>
__device__ __forceinline__ void rr2d_wait()
{
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"i"(N) : "memory");
}

// 16 B per lane from gsrc into LDS at byte address lds_dst + 16 lane (lds_dst wave-uniform)
__device__ __forceinline__ void rr2d_dma(const double* gsrc, unsigned lds_dst)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

template <int MODE, int NR, bool UN, bool WR>
__global__ __launch_bounds__(WAVE* RR2D_WXMAX) void k_rr2d(Coef k, const double* __restrict__ v,
                                                           const double* __restrict__ f, const double* __restrict__ w,
                                                           double* __restrict__ ca, double* __restrict__ cb, int fnx,
                                                           int fny, int fnz, int64_t fldy, int64_t fldz, int cnx,
                                                           int cny, int cnz, int64_t cldy, int64_t cldz, int ZC, int zhi)
{
    constexpr int RR = 2 * NR + 1;                   // computed fine rows; v rows 0 .. RR+1 (0, RR+1: halo rows)
    constexpr int RROWS = rr2d_rows<MODE, NR, WR>(); // ring rows per slot (= DMA instructions per wave and step)
    constexpr int RV = 0, RH = RR, RF = RR + 2, RW = 2 * RR + 2; // first row of each operand in a slot
    constexpr int NSTORE = 2 * NR;                               // coarse stores per wave at an even step
    constexpr int NWAIT = RROWS + NSTORE;                        // VMEM operations younger than the awaited plane's
    static_assert(NWAIT <= 63, "vmcnt field");
    extern __shared__ double ring[]; // [slot][row][WX * 128 doubles]; then re, ve
    const int lane = threadIdx.x;
    const int wx = __builtin_amdgcn_readfirstlane(threadIdx.y);
    const int WX = blockDim.y;
    const int RS = WX * 2 * WAVE; // doubles per ring row
    double* re = ring + RR2D_SLOTS * RROWS * RS; // r(2X+1) edges: [parity][1 + wave][row]
    double* ve = re + 2 * (RR2D_WXMAX + 2) * RR;  // prologue v edges: [1 + wave][side][row]
    const int tid = lane + WAVE * wx;
    for (int i = tid; i < 2 * (RR2D_WXMAX + 2) * RR + (RR2D_WXMAX + 2) * 2 * RR; i += WAVE * WX) re[i] = 0.0;
    const int64_t tile = xcd_tile(blockIdx.x + (int64_t)gridDim.x * blockIdx.y, (int64_t)gridDim.x * gridDim.y);
    const int Y = 1 + NR * (int)(tile % gridDim.x);
    const int Zb = 1 + (int)(tile / gridDim.x) * ZC, Ze = min(Zb + ZC - 1, cnz);
    const int X = 1 + wx * WAVE + lane;
    const int x = 2 * X - 1, xl = min(x, fnx + 1);
    const bool okx0 = x <= fnx, okx1 = x + 1 <= fnx;
    int64_t roff[RR + 2];
    bool rowc[RR + 2];
#pragma unroll
    for (int j = 0; j < RR + 2; j++) {
        const int y = 2 * Y - 2 + j;
        roff[j] = (int64_t)min(max(y, 0), fny + 1) * fldy;
        rowc[j] = y >= 1 && y <= fny;
    }
    auto at = [&](const double* b, int j, int p) {
        return b + xl + roff[j] + (int64_t)min(max(p, 0), fnz + 1 + zhi) * fldz;
    };
    typedef __attribute__((address_space(3))) double* lds_dp;
    const unsigned lbase = (unsigned)(uintptr_t)(lds_dp)ring;
    // this wave's 1 KB of ring row r of slot s, as an LDS byte address (wave-uniform)
    auto dst = [&](int s, int r) {
        return (unsigned)__builtin_amdgcn_readfirstlane((int)(lbase + 8u * (unsigned)((s * RROWS + r) * RS + wx * 2 * WAVE)));
    };
    // the operand rows of fine plane p into slot s
    auto dma_plane = [&](int s, int p) {
#pragma unroll
        for (int j = 0; j < RR; j++) rr2d_dma(at(v, j + 1, p + 1), dst(s, RV + j));
        rr2d_dma(at(v, 0, p), dst(s, RH));
        rr2d_dma(at(v, RR + 1, p), dst(s, RH + 1));
#pragma unroll
        for (int j = 0; j < RR; j++) rr2d_dma(at(f, j + 1, p), dst(s, RF + j));
        if constexpr (WR) {
#pragma unroll
            for (int j = 0; j < RR; j++) rr2d_dma(at(w, j + 1, p), dst(s, RW + j));
        }
    };
    auto row_at = [&](int s, int r) { return ring + (s * RROWS + r) * RS; };
    auto lds2 = [&](int s, int r) { return *reinterpret_cast<const double2*>(row_at(s, r) + wx * 2 * WAVE + 2 * lane); };
    double* sink = gs_rr2d_sink;

    // r = f - A v on fine plane p (k_rr2's resid: same expression, same term order; 0 outside the interior), with the
    // plane's 2 RR divisions by h^2 batched behind one range branch (div_hh_n: the same quotients bit for bit) — at
    // one wave per SIMD a branch per point would expose every point's latency
    auto resid = [&](const double2 (&Vm)[RR], const double2 (&Vc)[RR], const double2 (&H)[2], const double2 (&Vp)[RR],
                     const double2 (&F)[RR], const double2 (&W)[RR], const double (&CL)[RR], const double (&CR)[RR], int p,
                     double2 (&R)[RR]) {
        const bool pin = p >= 1 && (p <= fnz || (zhi && p == fnz + 1));
        double q[2 * RR];
#pragma unroll
        for (int j = 0; j < RR; j++) {
            const double2 c = Vc[j];
            const double2 ym = j == 0 ? H[0] : Vc[j - 1], yp = j == RR - 1 ? H[1] : Vc[j + 1];
            const double xm0 = lane_from_left<true>(c.y, CL[j]);
            const double xp1 = lane_from_right<true>(c.x, CR[j]);
            q[2 * j] = stencil_sum<UN>(k, c.x, c.y, xm0, yp.x, ym.x, Vp[j].x, Vm[j].x);
            q[2 * j + 1] = stencil_sum<UN>(k, c.y, xp1, c.x, yp.y, ym.y, Vp[j].y, Vm[j].y);
        }
        div_hh_n(k, q);
#pragma unroll
        for (int j = 0; j < RR; j++) {
            const double w0 = newtonish(MODE) ? W[j].x : 0.0, w1 = newtonish(MODE) ? W[j].y : 0.0;
            const double a0 = op_finish<MODE>(k, q[2 * j], Vc[j].x, w0);
            const double a1 = op_finish<MODE>(k, q[2 * j + 1], Vc[j].y, w1);
            const bool ok = pin && rowc[j + 1];
            R[j] = make_double2((ok && okx0) ? F[j].x - a0 : 0.0, (ok && okx1) ? F[j].y - a1 : 0.0);
        }
    };

    // prologue: the window v(p0 - 1), v(p0) (p0 = 2Zb - 1) by ordinary loads, v(p0)'s wave-edge columns through LDS
    const int p0 = 2 * Zb - 1;
    double2 Vm[RR], V0[RR];
    double CL0[RR], CR0[RR];
#pragma unroll
    for (int j = 0; j < RR; j++) {
        Vm[j] = ld2(at(v, j + 1, p0 - 1));
        V0[j] = ld2(at(v, j + 1, p0));
    }
    __syncthreads(); // (the zeroed re / ve)
    if (lane == 0) {
#pragma unroll
        for (int j = 0; j < RR; j++) ve[((wx + 1) * 2 + 0) * RR + j] = V0[j].x;
    }
    if (lane == WAVE - 1) {
#pragma unroll
        for (int j = 0; j < RR; j++) ve[((wx + 1) * 2 + 1) * RR + j] = V0[j].y;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RR; j++) {
        CL0[j] = uniform_d(ve[(wx * 2 + 1) * RR + j]);
        CR0[j] = uniform_d(ve[((wx + 2) * 2 + 0) * RR + j]);
    }
    // (every ordinary load above is complete: the ve writes needed them)
    dma_plane(p0 % RR2D_SLOTS, p0);
    dma_plane((p0 + 1) % RR2D_SLOTS, p0 + 1);
#pragma unroll
    for (int i = 0; i < NSTORE; i++) // the store group step p0's count expects (volatile: never merged or dropped)
        *reinterpret_cast<volatile double*>(sink + (i & 1) * WAVE + lane) = 0.0;

    double2 Ra[RR], Rb[RR], Rc[RR]; // r of planes p-3, p-2, p-1 entering step p
    double Na[RR], Nb[RR];          // r(2X+1) of planes p-3, p-2
#pragma unroll
    for (int j = 0; j < RR; j++) {
        Ra[j] = Rb[j] = Rc[j] = make_double2(0.0, 0.0);
        Na[j] = Nb[j] = 0.0;
    }
    const int pe = 2 * Ze + 2;
    auto step = [&](const int p, const bool even) {
        const int s = p % RR2D_SLOTS;
        rr2d_wait<NWAIT>();                              // plane p landed (every wave), slot p-1 read by every wave
        dma_plane((p + 2) % RR2D_SLOTS, p + 2);          // into the slot plane p-1 used
        double2 Vn[RR], H[2], F[RR], W[RR];
        double CLn[RR], CRn[RR], En[RR];
        // every LDS read of the step first, none under a branch (one wait for all of them): v(p+1)'s wave-edge
        // columns for the next step (from clamped columns, zero beyond the level's x-boundaries), r(2X+1) of plane
        // p-1 (its edge word written last step, visible past this step's barrier)
        const int cl = wx > 0 ? wx * 2 * WAVE - 1 : 0, cr = wx + 1 < WX ? (wx + 1) * 2 * WAVE : 0;
        const double* rprev = re + ((p - 1) & 1) * (RR2D_WXMAX + 2) * RR + (wx + 2) * RR;
#pragma unroll
        for (int j = 0; j < RR; j++) {
            Vn[j] = lds2(s, RV + j);
            F[j] = lds2(s, RF + j);
            if constexpr (WR) W[j] = lds2(s, RW + j);
            else if constexpr (MODE == GS_NEWTON_B) W[j] = make_double2(k.gamma, k.gamma); // (GS_NEWTON_G)
            else W[j] = make_double2(0.0, 0.0);
            CLn[j] = row_at(s, RV + j)[cl];
            CRn[j] = row_at(s, RV + j)[cr];
            En[j] = rprev[j];
        }
        H[0] = lds2(s, RH);
        H[1] = lds2(s, RH + 1);
#pragma unroll
        for (int j = 0; j < RR; j++) {
            CLn[j] = wx > 0 ? uniform_d(CLn[j]) : 0.0;
            CRn[j] = wx + 1 < WX ? uniform_d(CRn[j]) : 0.0;
        }
        double2 R[RR];
        resid(Vm, V0, H, Vn, F, W, CL0, CR0, p, R);
        double Nc[RR];
#pragma unroll
        for (int j = 0; j < RR; j++) Nc[j] = lane_from_right<true>(Rc[j].x, uniform_d(En[j]));
        // plane p's edge word, for the next step
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < RR; j++) re[(p & 1) * (RR2D_WXMAX + 2) * RR + (wx + 1) * RR + j] = R[j].x;
        }
        if (even) { // restriction of coarse plane Z = p / 2 - 1 from r of planes 2Z-1 .. 2Z+1 = p-3 .. p-1
            const int Z = p / 2 - 1;
#pragma unroll
            for (int i = 0; i < NR; i++) {
                double acc = 0.0;
#pragma unroll
                for (int a = -1; a <= 1; a++)
#pragma unroll
                    for (int b = -1; b <= 1; b++)
#pragma unroll
                        for (int c = -1; c <= 1; c++) {
                            const double wgt = 0.125 * ((2.0 - (a < 0 ? -a : a)) / 2.0) *
                                               ((2.0 - (b < 0 ? -b : b)) / 2.0) * ((2.0 - (c < 0 ? -c : c)) / 2.0);
                            const int j = 2 * i + b + 1;
                            const double2 rp = c < 0 ? Ra[j] : (c == 0 ? Rb[j] : Rc[j]);
                            const double rn = c < 0 ? Na[j] : (c == 0 ? Nb[j] : Nc[j]);
                            acc += wgt * (a < 0 ? rp.x : (a == 0 ? rp.y : rn));
                        }
                const bool ok = Z >= Zb && Z <= Ze && X <= cnx && Y + i <= cny;
                const int64_t q = X + (Y + i) * cldy + (int64_t)Z * cldz;
                double* pa = ok ? ca + q : sink + lane;
                double* pb = (ok && cb) ? cb + q : sink + WAVE + lane;
                *pa = acc;
                *pb = acc;
            }
        }
#pragma unroll
        for (int j = 0; j < RR; j++) {
            Vm[j] = V0[j];
            V0[j] = Vn[j];
            CL0[j] = CLn[j];
            CR0[j] = CRn[j];
            Ra[j] = Rb[j];
            Rb[j] = Rc[j];
            Rc[j] = R[j];
            Na[j] = Nb[j];
            Nb[j] = Nc[j];
        }
    };
    for (int p = p0; p <= pe; p += 2) {
        step(p, false);
        step(p + 1, true);
    }
    // drain: the last DMAs must land before the block's LDS can be reused by another block
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------
// Trilinear prolongation, closed form per fine point (the reference's inject + X, Y, Z passes,
// CpuSolver.cpp:240-290, combined in the same X -> Y -> Z order). Fine index P-1 is never written by
// the reference (stays 0) and coarse index Pc-1 is the zero boundary, so along each axis:
//   i even -> c(i/2);  i odd -> 0.5*c(i/2) + 0.5*c(i/2+1).
template <bool SUB>
__device__ __forceinline__ double coarse_at(const double* __restrict__ c, const double* __restrict__ sub, int64_t q)
{
    return SUB ? c[q] - sub[q] : c[q];
}

// (x, y, gz) are fine indices, gz global along z; the coarse field's local plane 0 is global cz0.
template <bool SUB>
__device__ __forceinline__ double prolong_value(const double* __restrict__ c, const double* __restrict__ sub, int x,
                                                int y, int gz, int64_t cldy, int64_t cldz, int cz0)
{
    const int cx = x >> 1, cy = y >> 1, cz = (gz >> 1) - cz0;
    const bool ox = x & 1, oy = y & 1, oz = gz & 1;
    auto X = [&](int jy, int jz) -> double {
        const int64_t q = cx + jy * cldy + (int64_t)jz * cldz;
        const double a = coarse_at<SUB>(c, sub, q);
        if (!ox) return a;
        const double b = coarse_at<SUB>(c, sub, q + 1);
        return 0.5 * a + 0.5 * b;
    };
    auto Y = [&](int jz) -> double {
        const double a = X(cy, jz);
        if (!oy) return a;
        const double b = X(cy + 1, jz);
        return 0.5 * a + 0.5 * b;
    };
    const double a = Y(cz);
    if (!oz) return a;
    const double b = Y(cz + 1);
    return 0.5 * a + 0.5 * b;
}

// Fused correction, two fine x-points per lane (x odd, x+1 even): one pair load / store of v, and
// per coarse row the two coarse values c(x>>1), c(x>>1 + 1) that both points interpolate from.
template <bool SUB>
__global__ __launch_bounds__(256) void k_prolong_add(const double* __restrict__ c, const double* __restrict__ sub,
                                                     double* __restrict__ fv, int fnx, int fny, int fnz, int64_t fldy,
                                                     int64_t fldz, int64_t cldy, int64_t cldz, int fz0, int cz0)
{
    const int t = blockIdx.x * 64 + threadIdx.x;
    const int x = 1 + 2 * t;
    const int y = 1 + blockIdx.y * 4 + threadIdx.y;
    const int z = 1 + blockIdx.z;
    if (x > fnx || y > fny) return;
    const int gz = z + fz0;
    const int cx = x >> 1, cy = y >> 1, cz = (gz >> 1) - cz0;
    const bool oy = y & 1, oz = gz & 1;
    // X pass: e0 at fine x (odd: average of c(cx), c(cx+1)), e1 at x+1 (even: injection of c(cx+1))
    auto X2 = [&](int jy, int jz, double& e0, double& e1) {
        const int64_t q = cx + jy * cldy + (int64_t)jz * cldz;
        const double a = coarse_at<SUB>(c, sub, q), b = coarse_at<SUB>(c, sub, q + 1);
        e0 = 0.5 * a + 0.5 * b;
        e1 = b;
    };
    // Y pass on top of X
    auto Y2 = [&](int jz, double& e0, double& e1) {
        double a0, a1;
        X2(cy, jz, a0, a1);
        if (!oy) {
            e0 = a0;
            e1 = a1;
            return;
        }
        double b0, b1;
        X2(cy + 1, jz, b0, b1);
        e0 = 0.5 * a0 + 0.5 * b0;
        e1 = 0.5 * a1 + 0.5 * b1;
    };
    double e0, e1;
    Y2(cz, e0, e1);
    if (oz) { // Z pass
        double g0, g1;
        Y2(cz + 1, g0, g1);
        e0 = 0.5 * e0 + 0.5 * g0;
        e1 = 0.5 * e1 + 0.5 * g1;
    }
    const int64_t p = x + y * fldy + (int64_t)z * fldz;
    if (x + 1 <= fnx) {
        const double2 v = ld2(fv + p);
        st2s<true>(fv + p, v.x + e0, v.y + e1);
    } else {
        fv[p] = fv[p] + e0;
    }
}

// The corrected iterate v + P v^2h on the four fine columns around every interior column-block
// boundary of the prolongation pair (k_tb2y XH + PRO): columns xb-2 .. xb+1 of the boundary at xb (the
// first column of the right block), rows 0..ny+1, local planes -1..nz+2 — what the blocks on either side
// read of the neighbour's columns. A point gets the correction where the pair's lanes correct it (x, y
// interior; the plane interior or a ghost plane of an internal slab side: pok) and keeps v elsewhere,
// with the reference's X, Y, Z pass arithmetic (prolong_value), so the strip holds bit for bit what the
// neighbour block's lanes compute in registers. Layout: es[((b * (nz + 4) + p + 1) * 4 + c) * (ny + 2) + y].
// The coarse field is indexed from the plane under fine local plane 0 (z0 even: local parities are global).
template <bool SUB>
__global__ __launch_bounds__(256) void k_pro_strip(const double* __restrict__ v, const double* __restrict__ c,
                                                   const double* __restrict__ sub, double* __restrict__ es, int nx,
                                                   int ny, int nz, int64_t ldy, int64_t ldz, int64_t cldy,
                                                   int64_t cldz, int bw, int zlo, int zhi)
{
    // four lanes per row (one per column), 64 rows per block: a wave's v load touches 16 rows' 32-B runs
    // and its coarse loads ~8 rows' lines (one thread per row and four columns, r03j: 159 us per 1024^3
    // launch, address-unit bound — every lane of a load on its own cache line)
    const int col = (int)threadIdx.x & 3;
    const int y = blockIdx.x * 64 + ((int)threadIdx.x >> 2);
    if (y > ny + 1) return;
    const int p = (int)blockIdx.y - 1;
    const int b = (int)blockIdx.z;
    const int x = 1 + (b + 1) * bw - 2 + col;
    const bool pok = (p >= 1 && p <= nz) || (zlo && p <= 0) || (zhi && p > nz);
    double val = v[x + (int64_t)y * ldy + (int64_t)p * ldz];
    if (pok && y >= 1 && y <= ny && x >= 1 && x <= nx) val = val + prolong_value<SUB>(c, sub, x, y, p, cldy, cldz, 0);
    es[(((int64_t)b * (nz + 4) + p + 1) * 4 + col) * (ny + 2) + y] = val;
}

// ---------------------------------------------------------------------------------------------
// Small levels (LINEAR, canonical stencil): a level's whole down-leg step or up-leg step in ONE launch
// of LDS-tiled blocks that recompute their halos instead of exchanging them. A 32^3 or 16^3 level is
// pure launch latency (~4.5 us per operator on a chip it cannot fill): the reference's pre-smoothing
// (2 sweeps), residual and restriction take one launch instead of three to five, the prolongation,
// correction and 2 post-smoothing sweeps one instead of three. A block owns a TS^3 tile of fine points
// (TS = 8: a 4^3 tile of coarse points) and evaluates every stage on the tile plus the halo the later
// stages read (v: 15^3 -> sweep 1: 13^3 -> sweep 2: 11^3 -> residual: 9^3 -> restriction), every point
// with the expression of the kernel it replaces (op_value / jacobi_update / the restriction's 27 terms
// in the reference's order / prolong_value), so every output is bit-identical to the unfused sequence.
// Points outside the level's interior keep their loaded value (a stored sweep leaves boundary values
// as they are) and have r = 0 (the reference never writes r there); loads are clamped to the padded
// array, whose clamped copies only ever feed such boundary points.
constexpr int TS = 8, TS_T = 1024; // 1024 threads: ~3 points per thread and stage (256: 12-14 us per launch, latency-bound)

// one Jacobi sweep over a tile: dst (edge dN) from src (edge dN + 2; dst i <-> src i + 1), f (and, NEWTON,
// the linearisation point w) from tiles of edge fN (dst i <-> f i + fo); global index of dst point 0: g0
template <int MODE, bool UN>
__device__ __forceinline__ void tile_sweep(const Coef& k, const double* src, double* dst, int dN, const double* F,
                                           const double* W, int fN, int fo, int gx0, int gy0, int gz0, int nx, int ny,
                                           int nz)
{
    const int sN = dN + 2, total = dN * dN * dN;
    for (int t = threadIdx.x; t < total; t += TS_T) {
        const int i = t % dN, j = (t / dN) % dN, l = t / (dN * dN);
        const int gx = gx0 + i, gy = gy0 + j, gz = gz0 + l;
        const int q = (i + 1) + sN * ((j + 1) + sN * (l + 1));
        const double c = src[q];
        double nv = c;
        if (gx >= 1 && gx <= nx && gy >= 1 && gy <= ny && gz >= 1 && gz <= nz) {
            const int qf = (i + fo) + fN * ((j + fo) + fN * (l + fo));
            const double w = newtonish(MODE) ? W[qf] : 0.0;
            const double a = op_value<MODE, UN>(k, c, src[q + 1], src[q - 1], src[q + sN], src[q - sN],
                                                 src[q + sN * sN], src[q - sN * sN], w);
            nv = jacobi_update<MODE>(k, c, F[qf] - a, w);
        }
        dst[t] = nv;
    }
}

// a tile of a padded field, clamped to the padded array (ZV: identically zero)
template <bool ZV>
__device__ __forceinline__ void tile_load(const double* __restrict__ g, double* dst, int N, int gx0, int gy0, int gz0,
                                          int nx, int ny, int nz, int64_t ldy, int64_t ldz)
{
    for (int t = threadIdx.x; t < N * N * N; t += TS_T) {
        if (ZV) {
            dst[t] = 0.0;
            continue;
        }
        const int i = t % N, j = (t / N) % N, l = t / (N * N);
        const int x = min(max(gx0 + i, 0), nx + 1), y = min(max(gy0 + j, 0), ny + 1), z = min(max(gz0 + l, 0), nz + 1);
        dst[t] = g[x + (int64_t)y * ldy + (int64_t)z * ldz];
    }
}

// pre-smoothing pair + residual + full weighting of a small level: v_out = S(S(v)) on the tile's fine
// points, coarse f = R(f - A v_out) on its coarse points (CpuSolver.cpp:88-99 with preSmoothing 2; ZV:
// v = 0, the coarse level's first sweeps after CpuSolver.cpp:100-101). MODE LINEAR, or NEWTON with the
// level's newtonV as w (the operator and the update linearised there, CpuSolver.cpp:63-66, :166-172).
template <int MODE, bool ZV, bool UN>
__global__ __launch_bounds__(TS_T) void k_tile_pre_rr(Coef k, const double* __restrict__ v, const double* __restrict__ f,
                                                      const double* __restrict__ w, double* __restrict__ vout,
                                                      double* __restrict__ cf, int nx, int ny, int nz, int64_t ldy,
                                                      int64_t ldz, int cnx, int cny, int cnz, int64_t cldy, int64_t cldz)
{
    constexpr int NV = TS + 7, N1 = TS + 5, N2 = TS + 3, NR = TS + 1, NF = TS + 5;
    constexpr int NW = newtonish(MODE) ? NF : 1;
    __shared__ double sv[NV * NV * NV], s1[N1 * N1 * N1], s2[N2 * N2 * N2], sf[NF * NF * NF], sw[NW * NW * NW];
    double* sr = sv; // the residual tile reuses v's storage once sweep 1 is done
    const int tx = 1 + TS * (int)blockIdx.x, ty = 1 + TS * (int)blockIdx.y, tz = 1 + TS * (int)blockIdx.z;
    tile_load<ZV>(v, sv, NV, tx - 3, ty - 3, tz - 3, nx, ny, nz, ldy, ldz);
    tile_load<false>(f, sf, NF, tx - 2, ty - 2, tz - 2, nx, ny, nz, ldy, ldz);
    if (newtonish(MODE)) tile_load<false>(w, sw, NF, tx - 2, ty - 2, tz - 2, nx, ny, nz, ldy, ldz);
    __syncthreads();
    tile_sweep<MODE, UN>(k, sv, s1, N1, sf, sw, NF, 0, tx - 2, ty - 2, tz - 2, nx, ny, nz);
    __syncthreads();
    tile_sweep<MODE, UN>(k, s1, s2, N2, sf, sw, NF, 1, tx - 1, ty - 1, tz - 1, nx, ny, nz);
    __syncthreads();
    // the tile's own fine points of v'' (interior only)
    for (int t = threadIdx.x; t < TS * TS * TS; t += TS_T) {
        const int i = t % TS, j = (t / TS) % TS, l = t / (TS * TS);
        const int x = tx + i, y = ty + j, z = tz + l;
        if (x <= nx && y <= ny && z <= nz)
            vout[x + (int64_t)y * ldy + (int64_t)z * ldz] = s2[(i + 1) + N2 * ((j + 1) + N2 * (l + 1))];
    }
    // r = f - A v'' on fine points tx .. tx + TS (the restriction's 3-point windows); 0 off the interior
    for (int t = threadIdx.x; t < NR * NR * NR; t += TS_T) {
        const int i = t % NR, j = (t / NR) % NR, l = t / (NR * NR);
        const int gx = tx + i, gy = ty + j, gz = tz + l;
        double r = 0.0;
        if (gx >= 1 && gx <= nx && gy >= 1 && gy <= ny && gz >= 1 && gz <= nz) {
            const int q = (i + 1) + N2 * ((j + 1) + N2 * (l + 1));
            const int qf = (i + 2) + NF * ((j + 2) + NF * (l + 2));
            const double c = s2[q];
            const double a = op_value<MODE, UN>(k, c, s2[q + 1], s2[q - 1], s2[q + N2], s2[q - N2], s2[q + N2 * N2],
                                                 s2[q - N2 * N2], newtonish(MODE) ? sw[qf] : 0.0);
            r = sf[qf] - a;
        }
        sr[t] = r;
    }
    __syncthreads();
    // coarse points X = (tx + 1) / 2 + 0..TS/2-1 (fine centre 2X = tx + 1 + 2u): the 27 terms in the
    // reference's order (CpuSolver.cpp:225-231)
    constexpr int TC = TS / 2;
    if (threadIdx.x < TC * TC * TC) {
        const int u = threadIdx.x % TC, o2 = (threadIdx.x / TC) % TC, o = threadIdx.x / (TC * TC);
        const int X = (tx + 1) / 2 + u, Y = (ty + 1) / 2 + o2, Z = (tz + 1) / 2 + o;
        if (X <= cnx && Y <= cny && Z <= cnz) {
            double acc = 0.0;
#pragma unroll
            for (int a = -1; a <= 1; a++)
#pragma unroll
                for (int b = -1; b <= 1; b++)
#pragma unroll
                    for (int c = -1; c <= 1; c++) {
                        const double wgt = 0.125 * ((2.0 - (a < 0 ? -a : a)) / 2.0) * ((2.0 - (b < 0 ? -b : b)) / 2.0) *
                                           ((2.0 - (c < 0 ? -c : c)) / 2.0);
                        acc += wgt * sr[(1 + 2 * u + a) + NR * ((1 + 2 * o2 + b) + NR * (1 + 2 * o + c))];
                    }
            cf[X + (int64_t)Y * cldy + (int64_t)Z * cldz] = acc;
        }
    }
}

// prolongation + correction + 2 post-smoothing sweeps of a small level: v_out = S(S(v + P c)) on the tile's
// fine points (CpuSolver.cpp:127-134 with the first two post-smoothing sweeps); MODE as above
template <int MODE, bool UN>
__global__ __launch_bounds__(TS_T) void k_tile_pro2(Coef k, const double* __restrict__ v, const double* __restrict__ c,
                                                    const double* __restrict__ f, const double* __restrict__ w,
                                                    double* __restrict__ vout, int nx, int ny, int nz, int64_t ldy,
                                                    int64_t ldz, int64_t cldy, int64_t cldz)
{
    constexpr int NU = TS + 4, N1 = TS + 2, NF = TS + 2;
    constexpr int NW = newtonish(MODE) ? NF : 1;
    __shared__ double su[NU * NU * NU], s1[N1 * N1 * N1], sf[NF * NF * NF], sw[NW * NW * NW];
    const int tx = 1 + TS * (int)blockIdx.x, ty = 1 + TS * (int)blockIdx.y, tz = 1 + TS * (int)blockIdx.z;
    for (int t = threadIdx.x; t < NU * NU * NU; t += TS_T) {
        const int i = t % NU, j = (t / NU) % NU, l = t / (NU * NU);
        const int gx = tx - 2 + i, gy = ty - 2 + j, gz = tz - 2 + l;
        const int x = min(max(gx, 0), nx + 1), y = min(max(gy, 0), ny + 1), z = min(max(gz, 0), nz + 1);
        double u = v[x + (int64_t)y * ldy + (int64_t)z * ldz];
        if (gx >= 1 && gx <= nx && gy >= 1 && gy <= ny && gz >= 1 && gz <= nz)
            u = u + prolong_value<false>(c, nullptr, gx, gy, gz, cldy, cldz, 0);
        su[t] = u;
    }
    tile_load<false>(f, sf, NF, tx - 1, ty - 1, tz - 1, nx, ny, nz, ldy, ldz);
    if (newtonish(MODE)) tile_load<false>(w, sw, NF, tx - 1, ty - 1, tz - 1, nx, ny, nz, ldy, ldz);
    __syncthreads();
    tile_sweep<MODE, UN>(k, su, s1, N1, sf, sw, NF, 0, tx - 1, ty - 1, tz - 1, nx, ny, nz);
    __syncthreads();
    for (int t = threadIdx.x; t < TS * TS * TS; t += TS_T) {
        const int i = t % TS, j = (t / TS) % TS, l = t / (TS * TS);
        const int gx = tx + i, gy = ty + j, gz = tz + l;
        if (gx > nx || gy > ny || gz > nz) continue;
        const int q = (i + 1) + N1 * ((j + 1) + N1 * (l + 1));
        const int qf = (i + 1) + NF * ((j + 1) + NF * (l + 1));
        const double cc = s1[q];
        const double wv = newtonish(MODE) ? sw[qf] : 0.0;
        const double a = op_value<MODE, UN>(k, cc, s1[q + 1], s1[q - 1], s1[q + N1], s1[q - N1], s1[q + N1 * N1],
                                             s1[q - N1 * N1], wv);
        vout[gx + (int64_t)gy * ldy + (int64_t)gz * ldz] = jacobi_update<MODE>(k, cc, sf[qf] - a, wv);
    }
}

// Unfused reference-shaped interpolate (whole padded fine array), used by parity tests.
__global__ __launch_bounds__(256) void k_interpolate(const double* __restrict__ c, double* __restrict__ e, int fPx,
                                                     int fPy, int fPz, int64_t fldy, int64_t fldz, int64_t cldy,
                                                     int64_t cldz)
{
    const int x = blockIdx.x * 64 + threadIdx.x;
    const int y = blockIdx.y * 4 + threadIdx.y;
    const int z = blockIdx.z;
    if (x >= fPx || y >= fPy) return;
    const int64_t p = x + y * fldy + (int64_t)z * fldz;
    if (x == fPx - 1 || y == fPy - 1 || z == fPz - 1) {
        e[p] = 0.0;
        return;
    }
    e[p] = prolong_value<false>(c, nullptr, x, y, z, cldy, cldz, 0);
}

// ---------------------------------------------------------------------------------------------
// Level-0 right-hand side, CpuGridData.cpp:7-12, 44-78 (same expression order).
__device__ __forceinline__ double rhs_f0(double x)
{
    return 100 * x * (x - 1.0) * x * (x - 1.0) * x * (x - 1.0) * x * (x - 1.0);
}
__device__ __forceinline__ double rhs_f2(double x)
{
    return 100.0 * 4.0 * (x - 1.0) * (x - 1.0) * x * x * (14.0 * x * x - 14.0 * x + 3);
}

__global__ __launch_bounds__(256) void k_rhs(double* __restrict__ f, int mode, double h, double gamma, int nx, int ny,
                                             int nz, int64_t z0, int64_t ldy, int64_t ldz)
{
    const int X = blockIdx.x * 64 + threadIdx.x; // padded indices
    const int Y = blockIdx.y * 4 + threadIdx.y;
    const int Z = blockIdx.z;
    if (X > nx + 1 || Y > ny + 1) return;
    const int64_t p = X + Y * ldy + (int64_t)Z * ldz;
    const int64_t Zg = Z + z0;
    if (mode == GS_LINEAR) {
        if (X < 1 || X > nx || Y < 1 || Y > ny || Z < 1 || Z > nz) return;
        const double x = (int)(X - 1) * h, y = (int)(Y - 1) * h, z = (int)(Zg - 1) * h;
        f[p] = -(rhs_f2(x) * rhs_f0(y) * rhs_f0(z) + rhs_f0(x) * rhs_f2(y) * rhs_f0(z) +
                 rhs_f0(x) * rhs_f0(y) * rhs_f2(z));
    } else {
        const double x = (int)X * h, y = (int)Y * h, z = (int)Zg * h;
        const double ux = x - x * x, uy = y - y * y, uz = z - z * z;
        f[p] = 2.0 * ((y - y * y) * (z - z * z) + (x - x * x) * (z - z * z) + (x - x * x) * (y - y * y)) +
               gamma * ux * uy * uz * exp(ux * uy * uz);
    }
}

// dst = src over n doubles (Vector3 copy-assignment): one dwordx4 per thread and iteration, both
// streams non-temporal (the 1 GB newtonF copy of a 512^3 Newton solve at the box's copy rate instead of
// hipMemcpyAsync's ~2.7 TB/s). head (0 or 1) leading elements bring both pointers to 16 B (a field's
// origin is 8 B past a 16-B boundary); they and an odd tail are copied by thread 0
__global__ __launch_bounds__(256) void k_copy(double* __restrict__ dst, const double* __restrict__ src, int64_t n,
                                              int head)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x, n2 = (n - head) / 2;
    const double* s = src + head;
    double* d = dst + head;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n2; i += stride) {
        const double2 t = ld2s<true>(s + 2 * i);
        st2s<true>(d + 2 * i, t.x, t.y);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (head) dst[0] = src[0];
        if ((n - head) & 1) dst[n - 1] = src[n - 1];
    }
}

// GS_NEWTON_B's linearisation factor (bfac_of) elementwise over n elements, dwordx4 streams when both arrays
// share an alignment (head: 0 or 1 leading element), else one per thread (-1)
__global__ __launch_bounds__(256) void k_bfac(double* __restrict__ b, const double* __restrict__ w, int64_t n,
                                              double gamma, int head)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x, t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (head < 0) {
        for (int64_t i = t0; i < n; i += stride) b[i] = bfac_of(gamma, w[i]);
        return;
    }
    const int64_t n2 = (n - head) / 2;
    for (int64_t i = t0; i < n2; i += stride) {
        const double2 t = ld2s<true>(w + head + 2 * i);
        st2s<true>(b + head + 2 * i, bfac_of(gamma, t.x), bfac_of(gamma, t.y));
    }
    if (t0 == 0) {
        if (head) b[0] = bfac_of(gamma, w[0]);
        if ((n - head) & 1) b[n - 1] = bfac_of(gamma, w[n - 1]);
    }
}

__global__ __launch_bounds__(256) void k_fill(double* __restrict__ dst, double value, int64_t n)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = value;
}

__global__ __launch_bounds__(256) void k_axpy(double* __restrict__ y, const double* __restrict__ x, double a,
                                              int64_t n)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
        if (a == 1.0) y[i] = y[i] + x[i];
        else if (a == -1.0) y[i] = y[i] - x[i];
        else y[i] = y[i] + a * x[i];
    }
}

// ---------------------------------------------------------------------------------------------
// The coarse end of the V-cycle in ONE launch of ONE workgroup (gs_coarse_cycle). A level of a few
// hundred points is pure launch latency per operator on a chip it cannot fill (~4.5 us a sweep);
// here the whole recursion of CpuSolver::vcycle below level lv[0] (CpuSolver.cpp:92-135) runs in one
// 1024-thread workgroup whose levels stay in L2, with a workgroup barrier between operators instead
// of a kernel boundary (the waves of a workgroup share one CU's L1, so the barrier's workgroup-scope
// fences order every store before the next operator's loads). Each point is computed by the
// expression of the per-operator kernel it replaces (k_generic KIND 0 / 1 / 2, k_restrict,
// k_prolong_add), so every field is bit-identical to the per-operator launch sequence.
constexpr int CC_T = 1024, CC_MAXLEV = 8;

struct CcLevel {
    double *v, *va, *f, *r, *rv, *w; // iterate, ping-pong partner, rhs, residual, restV (FAS), newtonV
    int64_t ldy, ldz;
    int nx, ny, nz, vz; // vz: the iterate is the zero iterate, not stored
    Coef k;
};
struct CcPlan {
    CcLevel L[CC_MAXLEV];
    int n, pre, post;
};

__device__ __forceinline__ int64_t cc_at(const CcLevel& L, int x, int y, int z)
{
    return x + y * L.ldy + (int64_t)z * L.ldz;
}

// dst[p] (and dst2[p]) = fn(x, y, z, p) for every interior point p of a level, x fastest, strided
// over the workgroup, B points per thread and pass: all B values are computed before any is stored,
// so a phase reading the field it writes (prolongation, f += A u) sees only old values.
template <int B, class F>
__device__ __forceinline__ void cc_map_b(const CcLevel& L, double* dst, double* dst2, F& fn)
{
    const int n = L.nx * L.ny * L.nz;
    for (int i0 = threadIdx.x; i0 < n; i0 += B * CC_T) {
        double val[B];
        int64_t q[B];
        bool ok[B];
#pragma unroll
        for (int b = 0; b < B; b++) {
            const int i = i0 + b * CC_T;
            ok[b] = i < n;
            const int ii = ok[b] ? i : i0; // a valid point; its value is discarded
            const int t = ii / L.nx, z = t / L.ny;
            const int x = 1 + ii - t * L.nx, y = 1 + t - z * L.ny;
            q[b] = cc_at(L, x, y, 1 + z);
            val[b] = fn(x, y, 1 + z, q[b]);
        }
#pragma unroll
        for (int b = 0; b < B; b++)
            if (ok[b]) {
                dst[q[b]] = val[b];
                if (dst2) dst2[q[b]] = val[b];
            }
    }
}
template <class F>
__device__ __forceinline__ void cc_map(const CcLevel& L, double* dst, double* dst2, F&& fn)
{
    cc_map_b<1>(L, dst, dst2, fn); // 2 points per pass measured no faster (the levels it runs are tiny)
}

// A(u) at p in config order (k_generic): the stencil sum, / h^2, the non-linear term; c = u(p),
// wv = w(p) (NEWTON). uz: u is the zero iterate (literal zeros, as k_generic's v == NULL).
template <int MODE>
__device__ __forceinline__ double cc_op(const Coef& k, const double* __restrict__ u, bool uz,
                                        const double* __restrict__ w, int64_t p, double& c, double& wv)
{
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 7; i++) s += k.s[i] * (uz ? 0.0 : u[p + k.off[i]]);
    s = div_hh(k, s);
    c = uz ? 0.0 : u[p];
    wv = newtonish(MODE) ? w[p] : 0.0;
    return op_finish<MODE>(k, s, c, wv);
}

template <int MODE>
__global__ __launch_bounds__(CC_T) void k_coarse_cycle(CcPlan P)
{
    unsigned alt = 0, zero = 0; // per level bit: the iterate is in va / is the unstored zero
    for (int l = 0; l < P.n; l++)
        if (P.L[l].vz) zero |= 1u << l;
    auto cur = [&](int l) { return ((alt >> l) & 1) ? P.L[l].va : P.L[l].v; };
    // v = 0 made real (HipSolver::materialize)
    auto materialize = [&](int l) {
        if (!((zero >> l) & 1)) return;
        const CcLevel& L = P.L[l];
        double* v = cur(l);
        cc_map(L, v, nullptr, [&](int, int, int, int64_t) { return 0.0; });
        __syncthreads();
        zero &= ~(1u << l);
    };
    // `sweeps` Jacobi sweeps, residual and update fused (k_generic KIND 0), ping-pong v <-> va
    auto smooth = [&](int l, int sweeps) {
        const CcLevel& L = P.L[l];
        if (sweeps == 0) materialize(l);
        for (int s = 0; s < sweeps; s++) {
            const bool uz = (zero >> l) & 1;
            const double* in = cur(l);
            double* out = ((alt >> l) & 1) ? L.v : L.va;
            cc_map(L, out, nullptr, [&](int, int, int, int64_t p) {
                double c, wv;
                const double a = cc_op<MODE>(L.k, in, uz, L.w, p, c, wv);
                const double r = L.f[p] - a;
                return jacobi_update<MODE>(L.k, c, r, wv);
            });
            __syncthreads();
            alt ^= 1u << l;
            zero &= ~(1u << l);
        }
    };
    // coarse interior of C <- 27-point full weighting of the fine field src of F (k_restrict)
    auto restrict_to = [&](const double* __restrict__ src, const CcLevel& F, double* ca, double* cb,
                           const CcLevel& C) {
        cc_map(C, ca, cb, [&](int x, int y, int z, int64_t) {
            const double* c0 = src + 2 * x + (int64_t)(2 * y) * F.ldy + (int64_t)(2 * z) * F.ldz;
            double acc = 0.0;
#pragma unroll
            for (int a = -1; a <= 1; a++)
#pragma unroll
                for (int b = -1; b <= 1; b++)
#pragma unroll
                    for (int c = -1; c <= 1; c++) {
                        const double wgt = 0.125 * ((2.0 - (a < 0 ? -a : a)) / 2.0) *
                                           ((2.0 - (b < 0 ? -b : b)) / 2.0) * ((2.0 - (c < 0 ? -c : c)) / 2.0);
                        acc += wgt * c0[a + b * F.ldy + c * F.ldz];
                    }
            return acc;
        });
    };

    // ---- down: pre-smoothing, f^2h = R(f - A v) [FAS: restV = v^2h = R v, f^2h += A(restV)] ----
    for (int l = 0; l + 1 < P.n; l++) {
        const CcLevel &F = P.L[l], &C = P.L[l + 1];
        smooth(l, P.pre);
        const double* u = cur(l);
        cc_map(F, F.r, nullptr, [&](int, int, int, int64_t p) { // residual (k_generic KIND 1)
            double c, wv;
            const double a = cc_op<MODE>(F.k, u, false, F.w, p, c, wv);
            return F.f[p] - a;
        });
        __syncthreads();
        restrict_to(F.r, F, C.f, nullptr, C);
        if (MODE == GS_NONLINEAR) restrict_to(u, F, C.rv, cur(l + 1), C);
        __syncthreads();
        if (MODE == GS_NONLINEAR) { // f += A(restV)  (k_generic KIND 2, ADD)
            cc_map(C, C.f, nullptr, [&](int, int, int, int64_t p) {
                double c, wv;
                const double a = cc_op<GS_NONLINEAR>(C.k, C.rv, false, nullptr, p, c, wv);
                return C.f[p] + a;
            });
            __syncthreads();
        }
    }
    // ---- the coarsest level: pre + post sweeps (CpuSolver.cpp:117) ----
    smooth(P.n - 1, P.pre + P.post);
    // ---- up: v^h += P(v^2h [- restV^2h]) (k_prolong_add), post-smoothing ----
    for (int l = P.n - 1; l > 0; l--) {
        const CcLevel &C = P.L[l], &F = P.L[l - 1];
        materialize(l);
        const double* cv = cur(l);
        double* fv = cur(l - 1);
        cc_map(F, fv, nullptr, [&](int x, int y, int z, int64_t p) {
            const double e = MODE == GS_NONLINEAR ? prolong_value<true>(cv, C.rv, x, y, z, C.ldy, C.ldz, 0)
                                                  : prolong_value<false>(cv, nullptr, x, y, z, C.ldy, C.ldz, 0);
            return fv[p] + e;
        });
        __syncthreads();
        smooth(l - 1, P.post);
    }
}

int launch_status()
{
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

bool bad_level(const gs_level* L)
{
    return !L || L->nx < 0 || L->ny < 0 || L->nz < 0 || L->ldy < L->nx + 2 || L->ldz < L->ldy * (L->ny + 2) ||
           L->nx > INT32_MAX / 2 || L->ny > INT32_MAX / 2 || L->nz > INT32_MAX / 2;
}

// Dispatch a stencil pass over (mode, kind) to the fast or the generic kernel.
// ---------------------------------------------------------------------------------------------
// Two fused Jacobi sweeps (temporal blocking): out = S(S(v)) reading v and f once and writing once
// (24 B per two lattice updates instead of 48). Wavefront along z: at step z the block computes
// sweep 1 at plane z — rows y0-1..y0+RY, i.e. one recomputed halo row per side — and sweep 2 at
// plane z-1 for rows y0..y0+RY-1. A block spans the whole x-row: WX waves of 128 columns whose
// outside columns (of v, and of the sweep-1 values) come from the neighbour waves through LDS, so
// nothing is recomputed along x. Where a sweep-1 point is a level boundary (x or y index 0 / n+1,
// z index 0 / nz+1 unless zlo / zhi says that side is an internal Z-slab boundary whose two ghost
// planes are current) its value is the boundary value itself, exactly as a stored sweep would leave
// it. Per point the arithmetic is the single sweep's, so the result is bit-identical to two
// gs_jacobi_sweep calls.
template <int MODE, int RY, int WXMAX, bool NT, bool NTF = NT, bool ZV = false>
__global__ __launch_bounds__(WAVE* WXMAX) void k_tb2(Coef k, const double* __restrict__ v,
                                                      const double* __restrict__ f, const double* __restrict__ w,
                                                      double* __restrict__ out, double* __restrict__ partials, int nx,
                                                      int ny, int nz, int64_t ldy, int64_t ldz, int ZC, int zlo,
                                                      int zhi, const double*, const double*, int, int, int, int64_t,
                                                      int64_t, const double*)
{
    __shared__ double red[WXMAX];
    double sumsq = 0.0; // r^2 of sweep 1's residual over the block's own points (partials != NULL)
    constexpr int NV = RY + 2;  // sweep-1 rows (j = 1..RY+2 <-> y0-1..y0+RY)
    constexpr int NE = NV + RY; // LDS edge values per wave side: v rows + sweep-1 rows
    // edge[parity][1 + wave][side][value]; slots 0 and WX+1 are virtual waves holding the x-boundary
    // columns, which this kernel takes to be zero (the reference's homogeneous Dirichlet boundary:
    // v's boundary cells are never written)
    __shared__ double edge[2][WXMAX + 2][2][NE];
    const int lane = threadIdx.x;
    const int wx = __builtin_amdgcn_readfirstlane(threadIdx.y);
    const int WX = blockDim.y;
    for (int i = threadIdx.x + threadIdx.y * WAVE; i < 2 * (WXMAX + 2) * 2 * NE; i += WAVE * WX)
        (&edge[0][0][0][0])[i] = 0.0;
    __syncthreads();
    const int x0 = 1 + wx * (2 * WAVE);
    const int x = x0 + 2 * lane;
    const int xl = min(x, nx + 1);
    const bool bx0 = x > nx, bx1 = x + 1 > nx;            // boundary / beyond columns
    const bool okx0 = x <= nx, okx1 = x + 1 <= nx;
    // XCD-aware order (cdna_hip_programming.md T1): hardware block b runs on XCD b % 8, so logical
    // tiles are dealt out in contiguous runs per XCD, y-tile fastest: the blocks an XCD runs at one
    // time are y-neighbours marching the same planes, and the halo rows one of them re-reads were
    // just fetched into that XCD's L2 by its neighbour.
    const int64_t tile = xcd_tile(blockIdx.x + (int64_t)gridDim.x * blockIdx.y, (int64_t)gridDim.x * gridDim.y);
    const int y0 = 1 + (int)(tile % gridDim.x) * RY;
    const int zb = 1 + (int)(tile / gridDim.x) * ZC;
    const int ze = min(zb + ZC - 1, nz);

    int64_t roff[RY + 4]; // rows y0-2 .. y0+RY+1
    bool rowc[RY + 4];    // row is a computable interior row
#pragma unroll
    for (int j = 0; j < RY + 4; j++) {
        const int y = y0 - 2 + j;
        roff[j] = (int64_t)min(max(y, 0), ny + 1) * ldy;
        rowc[j] = y >= 1 && y <= ny;
    }
    auto planeok = [&](int z) { return (z >= 1 && z <= nz) || (z == 0 && zlo) || (z == nz + 1 && zhi); };
    auto at = [&](const double* base, int j, int z) { return base + xl + roff[j] + (int64_t)z * ldz; };

    // Register window (rows j = 1..NV of the v planes; rows 0 and RY+3 only as halo pairs): Vp, Vc =
    // v at planes z-1, z; V1p, V1c = sweep-1 values at planes z-2, z-1; Fprev, Wprev = f, w at z-1.
    // What step z loads (v rows of plane z+2, f / w rows and the halo rows of plane z+1) goes into
    // slot ph of a two-slot ring and is consumed from there one step later before being moved on,
    // so every wait lands a full step of arithmetic after its load (loop unrolled by two).
    double2 Vp[NV], Vc[NV], VL[2][NV], FL[2][NV], WL[2][NV], HL[2][2];
    double2 V1p[RY], V1c[NV], Fprev[RY], Wprev[RY];
#pragma unroll
    for (int j = 0; j < NV; j++) V1c[j] = make_double2(0.0, 0.0);
#pragma unroll
    for (int j = 0; j < RY; j++) V1p[j] = make_double2(0.0, 0.0);
    // slot s <- plane z's f, w, halo rows and plane zv's v rows
    auto load_slot = [&](const int s, const int z, const int zv) {
#pragma unroll
        for (int j = 1; j <= NV; j++) {
            VL[s][j - 1] = ldv2<ZV>(at(v, j, zv));
            FL[s][j - 1] = ld2s<NTF>(at(f, j, z));
            if (newtonish(MODE)) WL[s][j - 1] = ld2(at(w, j, z));
        }
        HL[s][0] = ldv2<ZV>(at(v, 0, z));
        HL[s][1] = ldv2<ZV>(at(v, RY + 3, z));
    };
#pragma unroll
    for (int j = 1; j <= NV; j++) {
        Vp[j - 1] = ldv2<ZV>(at(v, j, zb - 2));
        Vc[j - 1] = ldv2<ZV>(at(v, j, zb - 1));
    }
    load_slot(1, zb - 1, zb);
    // Both halves always run (an odd step count ends with one step whose results are discarded) and
    // every load is unconditional (plane indices clamped into the padded range), so the slots keep
    // fixed registers around the loop.
    for (int z0 = zb - 1; z0 <= ze + 1; z0 += 2) {
#pragma unroll
        for (int ph = 0; ph < 2; ph++) {
            const int z = z0 + ph;
            const int cs = ph ^ 1; // slot holding plane z (and v of plane z+1)
            load_slot(ph, min(z + 1, nz + 1), min(z + 2, nz + 2));
            // ---- exchange the columns just outside each wave: v(z) rows 1..NV, sweep-1(z-1) rows 2..RY+1 ----
            if (lane == 0) {
#pragma unroll
                for (int j = 1; j <= NV; j++) edge[ph][wx + 1][0][j - 1] = Vc[j - 1].x;
#pragma unroll
                for (int j = 2; j <= RY + 1; j++) edge[ph][wx + 1][0][NV + j - 2] = V1c[j - 1].x;
            }
            if (lane == WAVE - 1) {
#pragma unroll
                for (int j = 1; j <= NV; j++) edge[ph][wx + 1][1][j - 1] = Vc[j - 1].y;
#pragma unroll
                for (int j = 2; j <= RY + 1; j++) edge[ph][wx + 1][1][NV + j - 2] = V1c[j - 1].y;
            }
            // LDS-only barrier: the outstanding prefetch must stay in flight across it
            __builtin_amdgcn_s_waitcnt(0xc07f); // lgkmcnt(0)
            __builtin_amdgcn_s_barrier();
            double CL[NE], CR[NE];
#pragma unroll
            for (int i = 0; i < NE; i++) {
                CL[i] = edge[ph][wx][1][i];     // wave wx-1 (slot 0: the zero x = 0 boundary)
                CR[i] = edge[ph][wx + 2][0][i]; // wave wx+1 (slot WX+1: the zero x = nx+1 boundary)
            }

            // ---- sweep 1 at plane z ----
            double2 V1n[NV];
            const bool pz = planeok(z);
#pragma unroll
            for (int j = 1; j <= NV; j++) {
                const double2 c = Vc[j - 1], zm = Vp[j - 1], zp = VL[cs][j - 1];
                const double2 ym = j == 1 ? HL[cs][0] : Vc[j - 2], yp = j == NV ? HL[cs][1] : Vc[j];
                const double xm0 = lane_from_left<true>(c.y, CL[j - 1]);
                const double xp1 = lane_from_right<true>(c.x, CR[j - 1]);
                const double wx0 = newtonish(MODE) ? WL[cs][j - 1].x : 0.0;
                const double wx1 = newtonish(MODE) ? WL[cs][j - 1].y : 0.0;
                const double a0 = op_value<MODE>(k, c.x, c.y, xm0, yp.x, ym.x, zp.x, zm.x, wx0);
                const double a1 = op_value<MODE>(k, c.y, xp1, c.x, yp.y, ym.y, zp.y, zm.y, wx1);
                const double r0 = FL[cs][j - 1].x - a0, r1 = FL[cs][j - 1].y - a1;
                const double n0 = jacobi_update<MODE>(k, c.x, r0, wx0);
                const double n1 = jacobi_update<MODE>(k, c.y, r1, wx1);
                if (partials && j >= 2 && j <= RY + 1 && z >= zb && z <= ze && rowc[j]) {
                    if (okx0) sumsq += r0 * r0;
                    if (okx1) sumsq += r1 * r1;
                }
                const bool keep = !pz || !rowc[j];
                V1n[j - 1] = make_double2((keep || bx0) ? c.x : n0, (keep || bx1) ? c.y : n1);
            }
            // ---- sweep 2 at plane z-1 ----
            if (z - 1 >= zb && z - 1 <= ze) {
                const int64_t zo = (int64_t)(z - 1) * ldz;
#pragma unroll
                for (int j = 2; j <= RY + 1; j++) {
                    const double2 c = V1c[j - 1], ym = V1c[j - 2], yp = V1c[j], zm = V1p[j - 2], zp = V1n[j - 1];
                    const double xm0 = lane_from_left<true>(c.y, CL[NV + j - 2]);
                    const double xp1 = lane_from_right<true>(c.x, CR[NV + j - 2]);
                    const double wx0 = newtonish(MODE) ? Wprev[j - 2].x : 0.0;
                    const double wx1 = newtonish(MODE) ? Wprev[j - 2].y : 0.0;
                    const double a0 = op_value<MODE>(k, c.x, c.y, xm0, yp.x, ym.x, zp.x, zm.x, wx0);
                    const double a1 = op_value<MODE>(k, c.y, xp1, c.x, yp.y, ym.y, zp.y, zm.y, wx1);
                    const double o0 = jacobi_update<MODE>(k, c.x, Fprev[j - 2].x - a0, wx0);
                    const double o1 = jacobi_update<MODE>(k, c.y, Fprev[j - 2].y - a1, wx1);
                    if (y0 - 2 + j <= ny) {
                        double* q = out + x + roff[j] + zo;
                        if (okx1) st2s<NT>(q, o0, o1);
                        else if (okx0) *q = o0;
                    }
                }
            }
            // ---- rotate (only registers whose loads were consumed above) ----
#pragma unroll
            for (int j = 0; j < RY; j++) {
                V1p[j] = V1c[j + 1];
                Fprev[j] = FL[cs][j + 1];
                if (newtonish(MODE)) Wprev[j] = WL[cs][j + 1];
            }
#pragma unroll
            for (int j = 0; j < NV; j++) {
                V1c[j] = V1n[j];
                Vp[j] = Vc[j];
                Vc[j] = VL[cs][j];
            }
        }
    }
    if (partials) {
        const double t = block_sum<WXMAX>(sumsq, red, WX);
        if (threadIdx.x == 0 && threadIdx.y == 0) partials[tile] = t;
    }
}

// The fused pair with two wave-rows per block ("tb2y"): the block is WX waves along x (the whole row)
// times 2 waves along y; the y-wave 0 owns output rows y0..y0+RY-1, the y-wave 1 rows
// y0+RY..y0+2RY-1. Between the two, the rows they need of each other (v of plane z and sweep-1 of
// plane z-1 at the shared edge) pass through LDS instead of being re-read and recomputed, so a block
// of 2RY output rows recomputes only ONE sweep-1 halo row per side and reads v rows y0-2..y0+2RY+1,
// f rows y0-1..y0+2RY: v 1 + 4/(2RY), f 1 + 2/(2RY) times the compulsory bytes before any L2 reuse
// (k_tb2 at RY rows per wave: 1 + 4/RY and 1 + 2/RY).
// Both y-waves run the same code on a local row index j = -1..RY+1: wave 0 maps j to y0-1+j, wave 1
// to the mirror image y0+2RY-j, so for both j = 0 is the recomputed halo row, j = 1..RY the own rows,
// j = RY the row published to the other wave, j = RY+1 the row received from it and j = -1 the one
// halo row of v loaded from memory. On wave 1 local j+1 is global y-1: the two y-neighbours are
// swapped back before the stencil sum, which keeps the reference's term order.
// PRO = 1 / 2: the input iterate is v + P(c) / v + P(c - sub) — the prolongation and correction of
// the V-cycle's up-leg (CpuSolver.cpp:121-132, gs_prolong_add) fused into the first post-smoothing
// pair, so the corrected iterate is never stored. The correction is added to every v value when it
// is consumed (the loads stay in flight as before): X-pass values of the two coarse planes under the
// current fine planes live in registers (W0, W1) and the next coarse plane is prefetched one step
// ahead; the z-chunk is even, so every fine plane's parity, hence its Y/Z combination, is static.
//
// XH (rows of more than 2 * WAVE * WX points): the row is split into column blocks of 2 * WAVE * WX
// points, one per block. The column just outside a block edge that is interior belongs to the
// neighbouring block; the edge wave computes what its LDS slot would hold there itself: v of plane z at
// that column (loads) and sweep 1 of plane z-1 at that column, evaluated lane-parallel one local row per
// lane (lane j <-> local row j, y-neighbours by lane shifts, x-neighbours loaded) with the same point
// expression, so every output is bit-identical to two gs_jacobi_sweep calls.
// TS (diagnostics only, gs_debug_pair_timestamps): es is a buffer of 4 doubles per tile that receives the
// block's start and end wall clock (100 MHz), its hardware block index and its HW_ID register
// WPE: waves per SIMD the register allocation must allow (0: the default, one; 4: <= 128 VGPRs, two 8-wave blocks per CU)
// FX (r06): every lane's two points lie inside the row (the host launches it where nx is a whole number of 128-point
// waves, 512-point column blocks for XH): the per-lane range selects of the new values, the norm partials and the stores
// fold away — the same values from fewer VALU instructions per step
template <int MODE, int RY, int WXMAX, bool NT, bool NTF = false, bool ZV = false, bool SPEC = false, int PRO = 0,
          int PFD = 1, bool XH = false, bool UN = false, bool TS = false, int WPE = 0, bool FX = false>
__global__ __launch_bounds__(WAVE* WXMAX * 2, WPE > 0 ? WPE : 1) void k_tb2y(Coef k, const double* __restrict__ v,
                                                           const double* __restrict__ f, const double* __restrict__ w,
                                                           double* __restrict__ out, double* __restrict__ partials,
                                                           int nx, int ny, int nz, int64_t ldy, int64_t ldz, int ZC,
                                                           int zlo, int zhi, const double* __restrict__ pc,
                                                           const double* __restrict__ ps, int cnx, int cny, int cnz,
                                                           int64_t cldy, int64_t cldz, const double* __restrict__ es)
{
    static_assert(PRO == 0 || (SPEC && !ZV && RY % 2 == 0), "fused prolongation: per-wave code, even RY");
    static_assert(!TS || (PRO == 0 && !XH), "timestamps: plain pairs (es carries the buffer)");
    const uint64_t tstart = TS ? wall_clock64() : 0;
    static_assert(!XH || ((PRO == 0 || MODE == GS_LINEAR || newtonish(MODE)) && RY + 2 <= WAVE),
                  "column blocks: every pair, LINEAR / NEWTON prolongation pairs");
    constexpr int NV = RY + 1;  // sweep-1 rows j = 0..RY
    constexpr int NE = NV + RY; // x-edge values per wave side: v rows 0..RY, sweep-1 rows 1..RY
    __shared__ double red[2 * WXMAX];
    // x-edges: [parity][y-wave][1 + x-wave][side][value]; x-wave slots 0 and WX+1 are the zero
    // x-boundary columns (the reference's homogeneous Dirichlet boundary)
    __shared__ double edge[2][2][WXMAX + 2][2][NE];
    // y-edge rows: [parity][y-wave][x-wave][v | sweep-1][lane]
    __shared__ double2 yrow[2][2][WXMAX][2][WAVE];
    const int lane = threadIdx.x;
    const int wy = __builtin_amdgcn_readfirstlane(threadIdx.z);
    const int WX = blockDim.y;
    // XH (Coef::swz): the mirrored y-wave row runs its x-waves rotated by two, so that the two waves a SIMD
    // hosts (hardware wave i -> SIMD i mod 4) are never both edge waves (the edge column's extra work)
    // (not in the prolongation pairs: there the rotation costs the LINEAR column-block form 3 VGPRs, 8-12 B
    // spilled per lane, where it fits 253 without)
    const int wx = __builtin_amdgcn_readfirstlane(XH && PRO == 0 && k.swz && wy && WX == 4 ? (threadIdx.y + 2) & 3
                                                                                            : threadIdx.y);
    const int tid = threadIdx.x + WAVE * (threadIdx.y + WX * threadIdx.z);
    for (int i = tid; i < 2 * 2 * (WXMAX + 2) * 2 * NE; i += WAVE * WX * 2) (&edge[0][0][0][0][0])[i] = 0.0;
    __syncthreads();
    const int64_t tile = xcd_tile(blockIdx.x + (int64_t)gridDim.x * blockIdx.y, (int64_t)gridDim.x * gridDim.y);
    // XH: column blocks fastest (the two edges a pair of neighbours share are read on one XCD)
    const int BW = 2 * WAVE * WX; // columns per block
    const int nh = XH ? (nx + BW - 1) / BW : 1;
    const int hx = XH ? (int)((tile % gridDim.x) % nh) : 0;
    const int xb = 1 + hx * BW;
    const int x0 = xb + wx * (2 * WAVE);
    const int x = x0 + 2 * lane;
    const int xl = min(x, nx + 1);
    const bool bx0 = !FX && x > nx, bx1 = !FX && x + 1 > nx;
    const bool okx0 = FX || x <= nx, okx1 = FX || x + 1 <= nx;
    const int y0 = 1 + (int)((tile % gridDim.x) / nh) * (2 * RY);
    const int zb = 1 + (int)(tile / gridDim.x) * ZC;
    const int ze = min(zb + ZC - 1, nz);
    const bool mir = wy != 0;
    auto yof = [&](int j) { return mir ? y0 + 2 * RY - j : y0 - 1 + j; };

    int64_t roff[RY + 2]; // local rows j = -1..RY at index j+1
    bool rowc[RY + 2];
#pragma unroll
    for (int j = -1; j <= RY; j++) {
        const int y = yof(j);
        roff[j + 1] = (int64_t)min(max(y, 0), ny + 1) * ldy;
        rowc[j + 1] = y >= 1 && y <= ny;
    }
    auto planeok = [&](int z) { return (z >= 1 && z <= nz) || (z == 0 && zlo) || (z == nz + 1 && zhi); };
    auto at = [&](const double* base, int j, int z) { return base + xl + roff[j + 1] + (int64_t)z * ldz; };
    // XH edge column xe (wave 0: left of the block, wave WX-1: right of it) when it is interior
    const bool eL = XH && wx == 0 && hx > 0;
    const bool eR = XH && wx == WX - 1 && xb + BW <= nx;
    const bool edg = eL || eR; // wave-uniform
    const int xe = eL ? xb - 1 : xb + BW;
    int64_t eroff = 0; // lane j <-> local row j = 0..RY+1
    bool erowc = false;
    if (XH) {
        const int y = yof(min(lane, RY + 1));
        eroff = (int64_t)min(max(y, 0), ny + 1) * ldy;
        erowc = y >= 1 && y <= ny;
    }
    auto eat = [&](const double* base, int dx, int z) { return base + (xe + dx) + eroff + (int64_t)z * ldz; };
    // XH + PRO: the edge column's corrected iterate v + P v^2h (columns xe-1..xe+1) comes from the strip
    // k_pro_strip wrote for this launch (layout there): [boundary][plane -1..nz+2][column xb-2..xb+1][row]
    const double* esr = es;
    if (XH && PRO != 0 && edg) {
        const int hb = eL ? hx - 1 : hx; // the block boundary the edge column lies at
        const int y = yof(min(lane, RY + 1));
        esr = es + (int64_t)hb * (nz + 4) * 4 * (ny + 2) + (eL ? 1 : 2) * (ny + 2) + min(max(y, 0), ny + 1);
    }
    auto sat = [&](int dx, int z) { return esr + ((int64_t)(z + 1) * 4 + dx) * (ny + 2); };

    // PFD: prefetch distance in plane steps. 1: two operand slots (this step's, the next one's in
    // flight); 2: four named slots, three live (this step's and the next two in flight), the z loop
    // unrolled by 4 so every slot index is static
    static_assert(PFD == 1 || PFD == 2, "prefetch distance 1 or 2");
    constexpr int NS = PFD == 2 ? 4 : 2, UNR = PFD == 2 ? 4 : 2;
    double2 Vp[NV], Vc[NV], VL[NS][NV], FL[NS][NV], WL[NS][NV], HL[NS];
    double2 V1p[RY], V1c[NV], Fprev[RY], Aprev[RY], Eprev[RY]; // Aprev, Eprev: NEWTON terms at z-1
    // YSH (GS_NEWTON_B plain pairs): the E slots (E = 1 there) carry the point's Jacobi reciprocal nb_recip(preFac + B),
    // formed in sweep 1 and reused by sweep 2 one plane step later — the same value, so bit-identical to nb_quot at
    // both sweeps (232-238 VGPRs, no spill): pair 0.806-0.829 vs 0.829-0.840 ms, Newton iteration 27.74-28.07 vs
    // 28.21-28.48 ms (r05t; in the prolongation pairs too: the same Newton time, 255 VGPRs, and the two-x-wave
    // instance falls to one wave per SIMD, r05s)
    // (the zero-iterate pairs too, though it costs them their third wave per SIMD: 166 -> 177 VGPRs; without them
    // 28.54-28.81 vs 28.08-28.43 ms per Newton iteration, r05u)
    // (and the four-x-wave prolongation pair, 255 VGPRs, no spill: 0.906-0.918 vs 0.935-0.943 ms per 512^3 launch,
    // Newton iteration 27.74-28.04 vs 27.99-28.25 ms, r05z; the two-x-wave instance of 256-point rows keeps
    // recomputing: at 255 VGPRs it would fall to one wave per SIMD, r05s)
    constexpr bool YSH = MODE == GS_NEWTON_B && !XH && (PRO == 0 || WXMAX > 2);
#ifdef GS_EXP_EFIELD
    double2 XL[NS][NV];
#endif
    // NEWTON with the fused prolongation: no room for Aprev / Eprev, so sweep 2 recomputes A from the
    // newtonV rows at z-1 and reads E = exp(w) from LDS (same expressions, same values)
    // NEWTON column blocks (XH) likewise: their edge-column state leaves no room for Aprev / Eprev / Fprev
    // (GS_NEWTON_B prolongation pairs keep them in registers: A = B, E = 1, 246 VGPRs without spill; 0.968-0.979 vs
    // 0.986-0.990 ms per 512^3 launch with the LDS state, profiles/r05/r05g_newton_b_norecomp_touch_ab.txt)
    constexpr bool RECOMP = newtonish(MODE) && ((PRO != 0 && MODE == GS_NEWTON) || XH);
    constexpr bool ELDS = RECOMP && MODE == GS_NEWTON; // E in LDS (GS_NEWTON_B: E = 1, A = B from wprev_l)
    constexpr bool WLDS = newtonish(MODE) && PRO != 0; // the coarse X-pass rows in LDS (prolongation pairs)
    // (Wprev, Fprev: sweep 2's newtonV / f rows at z-1, in LDS like the coarse rows below)
    __shared__ double2 wprev_l[RECOMP ? RY : 1][RECOMP ? 2 * WXMAX : 1][RECOMP ? WAVE : 1];
    __shared__ double2 fprev_l[RECOMP ? RY : 1][RECOMP ? 2 * WXMAX : 1][RECOMP ? WAVE : 1];
    // exp(w) of sweep 1's own rows, by plane parity: sweep 2 reads the previous plane's (each lane its own
    // values, no barrier) instead of evaluating exp a second time (+32 KB: 148 KB, one block per CU as before)
    __shared__ double2 eprev_l[ELDS ? 2 : 1][ELDS ? RY : 1][ELDS ? 2 * WXMAX : 1][ELDS ? WAVE : 1];
#pragma unroll
    for (int j = 0; j < NV; j++) V1c[j] = make_double2(0.0, 0.0);
#pragma unroll
    for (int j = 0; j < RY; j++) V1p[j] = make_double2(0.0, 0.0);
    // XH edge column: v at plane z+1 (EA), its x-neighbours (EXm, EXp) and f at plane z, per slot;
    // EP / EC: v at planes z-1 / z; ES1c: sweep 1 at plane z-1
    // NEWTON (EPK): the five edge values of a step share ONE register per slot: lane 8 f + r holds field f
    // (0 v or the corrected v at plane z+1, 1 / 2 its x-neighbours at plane z, 3 f, 4 newtonV) of local row r,
    // and the edge computation takes them with lane permutes. The prefetch distance stays one step, at 2
    // VGPRs per slot instead of 10 (the NEWTON column-block pairs spilled with five slot arrays)
    constexpr bool EPK = XH && newtonish(MODE);
    constexpr int NES = (XH && !EPK) ? NS : 1;
    double EA[NES], EXm[NES], EXp[NES], EF[NES], EP = 0.0, EC = 0.0, ES1c = 0.0;
    double EPS[EPK ? NS : 1]; // EPK: the packed slots
    auto load_edge = [&](const int s, const int z, const int zv) {
        if constexpr (PRO != 0) {
            EA[s] = *sat(0, zv);
            EXm[s] = *sat(-1, z);
            EXp[s] = *sat(1, z);
        } else {
            EA[s] = ldv1<ZV>(eat(v, 0, zv));
            EXm[s] = ldv1<ZV>(eat(v, -1, z));
            EXp[s] = ldv1<ZV>(eat(v, 1, z));
        }
        EF[s] = *eat(f, 0, z);
    };
    // EPK: lane 8 f + r's row offset (row r = 0..7 clamped to the edge rows 0..RY+1) and field f
    const int pfld = EPK ? lane >> 3 : 0;
    int64_t proff = 0;
    const double* psr = es;
    if constexpr (EPK) {
        const int y = yof(min(lane & 7, RY + 1));
        proff = (int64_t)min(max(y, 0), ny + 1) * ldy;
        if (PRO != 0 && edg) {
            const int hb = eL ? hx - 1 : hx;
            psr = es + (int64_t)hb * (nz + 4) * 4 * (ny + 2) + (eL ? 1 : 2) * (ny + 2) + min(max(y, 0), ny + 1);
        }
    }
    auto load_packed = [&](const int s, const int z, const int zv) {
        const int dx = pfld == 1 ? -1 : (pfld == 2 ? 1 : 0);
        const int zz = pfld == 0 ? zv : z;
        double val = 0.0;
        if (pfld <= 2) {
            if constexpr (PRO != 0) val = psr[((int64_t)(zz + 1) * 4 + dx) * (ny + 2)];
            else if constexpr (!ZV) val = v[(xe + dx) + proff + (int64_t)zz * ldz];
        } else if (pfld == 3) {
            val = f[xe + proff + (int64_t)z * ldz];
        } else if (pfld == 4) {
            val = (MODE == GS_NEWTON_B && k.bconst) ? k.gamma : w[xe + proff + (int64_t)z * ldz];
        }
        EPS[s] = val;
    };
    // field fl of this lane's edge row from packed slot s (a lane permute; every lane of the wave active)
    auto efld = [&](const int s, const int fl) { return __shfl(EPS[s], fl * 8 + (lane & 7), WAVE); };
    // GRP (LINEAR plain pairs, r06): a step's loads grouped by field and plane, rows ascending — v's halo row and rows
    // 0..RY, then f's rows — instead of row by row alternating between the two streams: pair 0.5831-0.5998 vs
    // 0.5935-0.6013 ms per 512^3 launch, 5 of 6 interleaved rounds faster (profiles/r06/r06v_pair_load_order_ab.txt,
    // r06u); the NEWTON pairs and every prolongation pair measured slower with it (r06u / r06v) and keep the row order
    constexpr bool GRP = MODE == GS_LINEAR && PRO == 0;
    auto load_slot = [&](const int s, const int z, const int zv) {
        if constexpr (GRP) {
            HL[s] = ldv2<ZV>(at(v, -1, z));
#pragma unroll
            for (int j = 0; j < NV; j++) VL[s][j] = ldv2<ZV>(at(v, j, zv));
#pragma unroll
            for (int j = 0; j < NV; j++) FL[s][j] = ld2s<NTF>(at(f, j, z));
        } else {
#pragma unroll
            for (int j = 0; j < NV; j++) {
                VL[s][j] = ldv2<ZV>(at(v, j, zv));
                FL[s][j] = ld2s<NTF>(at(f, j, z));
                if (MODE == GS_NEWTON_B && k.bconst) WL[s][j] = make_double2(k.gamma, k.gamma);
                else if (newtonish(MODE)) WL[s][j] = ld2(at(w, j, z));
#ifdef GS_EXP_EFIELD
                if (MODE == GS_NEWTON) XL[s][j] = ld2(at(w, j, z) + k.efoff);
#endif
            }
            HL[s] = ldv2<ZV>(at(v, -1, z));
        }
        if constexpr (XH && !EPK) {
            if (edg) load_edge(s, z, zv);
        }
        if constexpr (EPK) {
            if (edg) load_packed(s, z, zv);
        }
    };
#pragma unroll
    for (int j = 0; j < NV; j++) {
        Vp[j] = ldv2<ZV>(at(v, j, zb - 2));
        Vc[j] = ldv2<ZV>(at(v, j, zb - 1));
    }
    if (XH && edg) {
        EP = PRO != 0 ? *sat(0, zb - 2) : ldv1<ZV>(eat(v, 0, zb - 2));
        EC = PRO != 0 ? *sat(0, zb - 1) : ldv1<ZV>(eat(v, 0, zb - 1));
    }
    // ---- fused prolongation (PRO): coarse rows cyb .. cyb+NCR-1 lie under the wave's fine rows ----
    constexpr int NCR = RY / 2 + 2;
    // RBDPP (NEWTON column blocks, where every VGPR counts): b = c(cx+1) is the next lane's a (one DPP shift; lane
    // 63 takes the next wave's first column as a wave-uniform load), so a is clamped to cnx+1 instead of cnx —
    // the same b for every lane, a different a only for lanes past the row's end, which correct nothing
    constexpr bool RBDPP = newtonish(MODE) && XH && PRO == 1;
    const int cxl = min(x >> 1, max(RBDPP ? cnx + 1 : cnx, 0)); // the lane's coarse column (fine pair x odd, x+1 even)
    const int cxe = min((x0 >> 1) + WAVE, cnx + 1);             // RBDPP: lane 63's b column
    const int cyb = mir ? ((y0 - 1) >> 1) + RY / 2 : ((y0 - 1) >> 1) - 1;
    int64_t crow[NCR];
#pragma unroll
    for (int r = 0; r < NCR; r++) crow[r] = (int64_t)min(max(cyb + r, 0), cny + 1) * cldy;
    double2 W0[NCR], W1[NCR], Wm[NCR]; // X-pass values of coarse planes K, K+1 (Wm: K-1, first step)
    // HALF: the same rows times 0.5, the product every Y and Z pass of the reference takes of them first
    // (0.5 * fine(y-1) + 0.5 * fine(y+1) with fine(y+-1) an X-pass value; 0.5 * fine(z) + 0.5 * fine(z+2)
    // with fine(z), fine(z+2) X-pass values on even rows): formed once per coarse row instead of at every
    // fine point that reads it — the same products, so the same bits
    constexpr bool HALF = !WLDS;
    double2 H0[HALF ? NCR : 1], H1[HALF ? NCR : 1], Hm[HALF ? NCR : 1];
    // NEWTON (RECOMP): the X-pass rows of planes K, K+1 live in LDS, slot wsl / wsl^1 — each lane
    // reads back only what it wrote, so no barrier; this keeps the variant inside 256 VGPRs
    __shared__ double2 wlds[WLDS ? 2 : 1][WLDS ? 2 * WXMAX : 1][WLDS ? NCR : 1][WLDS ? WAVE : 1];
    int wsl = 0;
    const int wid_l = WLDS ? wx + WX * wy : 0;
    // coarse X-pass row r of plane slot s (0: K, 1: K+1, 2: K-1 on the first step)
    auto wget = [&](int s, int r) -> double2 {
        if (s == 2) return Wm[r];
        if constexpr (WLDS) return wlds[s ^ wsl][wid_l][r][lane];
        else return s == 0 ? W0[r] : W1[r];
    };
    auto hget = [&](int s, int r) -> double2 { return s == 2 ? Hm[HALF ? r : 0] : (s == 0 ? H0[HALF ? r : 0] : H1[HALF ? r : 0]); };
    double RA[NCR], RB[RBDPP ? 1 : NCR], RE[RBDPP ? NCR : 1], SA[NCR], SB[NCR]; // raw c (and sub) of plane K+2, in flight
    auto craw = [&](int cz) {
        // coarse planes -1 .. cnz+2 exist in the layout; only those under corrected fine planes matter
        const int64_t zp = (int64_t)min(max(cz, -1), cnz + 2) * cldz, zo = zp + cxl;
#pragma unroll
        for (int r = 0; r < NCR; r++) {
            RA[r] = pc[zo + crow[r]];
            if constexpr (RBDPP) RE[r] = pc[zp + crow[r] + cxe];
            else RB[r] = pc[zo + crow[r] + 1];
            if (PRO == 2) {
                SA[r] = ps[zo + crow[r]];
                SB[r] = ps[zo + crow[r] + 1];
            }
        }
    };
    // X pass of gs_prolong_add: e(x odd) = 0.5 a + 0.5 b, e(x+1 even) = b, a / b = c(cx) / c(cx+1)
    auto xpass = [&](int s) {
#pragma unroll
        for (int r = 0; r < NCR; r++) {
            const double a = PRO == 2 ? RA[r] - SA[r] : RA[r];
            const double b = RBDPP ? lane_from_right<true>(RA[r], RE[RBDPP ? r : 0])
                                   : (PRO == 2 ? RB[r] - SB[r] : RB[RBDPP ? 0 : r]);
            const double2 X = make_double2(0.5 * a + 0.5 * b, b);
            if constexpr (HALF) {
                const double2 Hh = make_double2(0.5 * X.x, 0.5 * X.y);
                if (s == 2) Hm[r] = Hh;
                else if (s == 0) H0[r] = Hh;
                else H1[r] = Hh;
            }
            if (s == 2) Wm[r] = X;
            else if constexpr (WLDS) wlds[s ^ wsl][wid_l][r][lane] = X;
            else if (s == 0) W0[r] = X;
            else W1[r] = X;
        }
    };
    // the correction of local row j on a plane whose coarse neighbours are Wa (and Wb when the fine
    // plane is odd), Y pass then Z pass; added where the fine point is interior
    auto correct = [&](double2& val, int j, bool zodd, bool zin, int sa, int sb, auto mirc) {
        constexpr bool M = decltype(mirc)::get();
        const int u = M ? 2 * RY + 1 - j : j + 2; // fine row = 2 (coarse base) + u
        const int ri = M ? (u >> 1) - RY / 2 : (u >> 1);
        const bool yodd = u & 1;
        auto ypass = [&](int s) {
            const double2 X0 = wget(s, ri);
            if (!yodd) return X0;
            const double2 X1 = wget(s, ri + 1);
            return make_double2(0.5 * X0.x + 0.5 * X1.x, 0.5 * X0.y + 0.5 * X1.y);
        };
        double2 e;
        if constexpr (HALF) {
            auto hsum = [](double2 p, double2 q) { return make_double2(p.x + q.x, p.y + q.y); };
            if (!zodd) {
                e = yodd ? hsum(hget(sa, ri), hget(sa, ri + 1)) : wget(sa, ri);
            } else if (!yodd) {
                e = hsum(hget(sa, ri), hget(sb, ri));
            } else {
                const double2 ea = hsum(hget(sa, ri), hget(sa, ri + 1)), eb = hsum(hget(sb, ri), hget(sb, ri + 1));
                e = make_double2(0.5 * ea.x + 0.5 * eb.x, 0.5 * ea.y + 0.5 * eb.y);
            }
        } else {
            e = ypass(sa);
            if (zodd) {
                const double2 g = ypass(sb);
                e = make_double2(0.5 * e.x + 0.5 * g.x, 0.5 * e.y + 0.5 * g.y);
            }
        }
        if (zin && rowc[j + 1]) {
            if (okx0) val.x = val.x + e.x;
            if (okx1) val.y = val.y + e.y;
        }
    };
    // a fine plane gets the correction when it is interior or a ghost plane of an internal slab side
    auto pok = [&](int p) { return (p >= 1 && p <= nz) || (zlo && p <= 0) || (zhi && p > nz); };
    if (PRO) {
        const int m0 = (zb - 1) >> 1; // zb is odd: planes zb-2 = 2 m0 - 1, zb - 1 = 2 m0
        craw(m0 - 1);
        xpass(2);
        craw(m0);
        xpass(0);
        craw(m0 + 1);
        xpass(1);
        auto pro_init = [&](auto mirc) {
#pragma unroll
            for (int j = 0; j < NV; j++) {
                correct(Vp[j], j, true, pok(zb - 2), 2, 0, mirc);
                correct(Vc[j], j, false, pok(zb - 1), 0, 0, mirc);
            }
        };
        if (mir) pro_init(BoolC<true>{});
        else pro_init(BoolC<false>{});
    }
    if (PFD == 1) {
        load_slot(1, zb - 1, zb);
    } else {
        load_slot(0, zb - 1, zb);
        load_slot(1, zb, zb + 1);
    }
    double sumsq = 0.0;
    for (int z0 = zb - 1; z0 <= ze + 1; z0 += UNR) {
#pragma unroll
        for (int ph4 = 0; ph4 < UNR; ph4++) {
            // the last two steps of a 4-step round are skipped past the chunk (uniform branch)
            if (UNR == 4 && ph4 == 2 && z0 + 2 > ze + 1) break;
            const int ph = ph4 & 1; // plane parity (z0 is even): LDS double buffers, PRO combinations
            const int z = z0 + ph4;
            const int cs = PFD == 1 ? ph ^ 1 : ph4; // slot holding this step's operands
            if (PFD == 1) load_slot(ph, min(z + 1, nz + 1), min(z + 2, nz + 2));
            else load_slot((ph4 + 2) & 3, min(z + 2, nz + 1), min(z + 3, nz + 2));
            if (PRO && ph == 0) craw((z >> 1) + 2); // consumed at the end of the next step
            // ---- publish: x-edge columns (v(z) rows 0..RY, sweep-1(z-1) rows 1..RY) and the y-edge row
            if (lane == 0) {
#pragma unroll
                for (int j = 0; j < NV; j++) edge[ph][wy][wx + 1][0][j] = Vc[j].x;
#pragma unroll
                for (int j = 1; j <= RY; j++) edge[ph][wy][wx + 1][0][NV + j - 1] = V1c[j].x;
            }
            if (lane == WAVE - 1) {
#pragma unroll
                for (int j = 0; j < NV; j++) edge[ph][wy][wx + 1][1][j] = Vc[j].y;
#pragma unroll
                for (int j = 1; j <= RY; j++) edge[ph][wy][wx + 1][1][NV + j - 1] = V1c[j].y;
            }
            yrow[ph][wy][wx][0][lane] = Vc[RY];
            yrow[ph][wy][wx][1][lane] = V1c[RY];
            // LDS-only barrier: the outstanding prefetch stays in flight across it
            GS_LDS_BARRIER(); // lgkmcnt(0), s_barrier
            double CL[NE], CR[NE];
            // VEDGE (r06: LINEAR plain and prolongation pairs on whole rows, the GS_NEWTON_B FX plain pair): the edge
            // values stay in the VGPRs the LDS broadcast read fills, and each DPP shift takes its edge as the old value
            // in place — no readfirstlane to SGPRs and no copy back to a VGPR per shift (20 fewer VALU instructions per
            // plane step, +20 VGPRs: 230 / 248 / 252, no spill). Pair 0.557-0.568 vs 0.574-0.583 ms, LINEAR prolongation
            // pair 0.652-0.661 vs 0.665-0.674 ms, Newton iteration 27.54-27.65 vs 27.65-28.04 ms (rotated rounds,
            // profiles/r06/r06ad_pair_vedge_ab.txt, r06ag_vedge_pro_newton_ab.txt); the other pairs keep them in SGPRs
            // (the extra VGPRs would spill or cost them a wave per SIMD)
            constexpr bool VEDGE = !XH && (MODE == GS_LINEAR || (MODE == GS_NEWTON_B && PRO == 0 && FX));
#pragma unroll
            for (int i = 0; i < NE; i++) { // wave-uniform: kept in SGPRs (VEDGE: VGPRs)
                if constexpr (VEDGE) {
                    CL[i] = edge[ph][wy][wx][1][i];
                    CR[i] = edge[ph][wy][wx + 2][0][i];
                } else {
                    CL[i] = uniform_d(edge[ph][wy][wx][1][i]);
                    CR[i] = uniform_d(edge[ph][wy][wx + 2][0][i]);
                }
            }
            const double2 vY = yrow[ph][wy ^ 1][wx][0][lane]; // v(z) at local row RY+1
            const double2 sY = yrow[ph][wy ^ 1][wx][1][lane]; // sweep-1(z-1) at local row RY+1
            if constexpr (XH) {
                // the edge column beyond an interior block edge: v(z) rows 0..RY, sweep-1(z-1) rows 1..RY
                if (edg) {
#pragma unroll
                    for (int i = 0; i < NE; i++) {
                        const double e = i < NV ? EC : ES1c;
                        const int ln = i < NV ? i : i - NV + 1;
                        const long long b = __double_as_longlong(e);
                        const int lo = __builtin_amdgcn_readlane((int)b, ln), hi = __builtin_amdgcn_readlane((int)(b >> 32), ln);
                        const double u = __longlong_as_double(((long long)(unsigned)hi << 32) | (unsigned)lo);
                        if (eL) CL[i] = u;
                        else CR[i] = u;
                    }
                }
            }

            // ---- the two sweeps; wave 1 (mirrored rows) runs its own copy of the code, so the swap of
            // its y-neighbours costs no selects ----
            double2 V1n[NV];
            double2 Acur[RY], Ecur[RY]; // NEWTON terms of sweep 1's own rows (-> Aprev / Eprev)
            const bool pz = planeok(z);
            double ES1n = 0.0;
            auto sweeps = [&](auto mirc) {
                const bool M = mirc.get();
                if constexpr (XH) {
                    // sweep 1 at plane z on the edge column, local row = lane (rows 1..RY are used)
                    if (edg) {
                        const double c = EC;
                        const double lm = lane_from_left<true>(EC, 0.0), lp = lane_from_right<true>(EC, 0.0);
                        const double ym = M ? lp : lm, yp = M ? lm : lp;
                        double nv;
                        // (zero iterate: q = +0 exactly, Coef::zq)
                        auto qe = [&] {
                            if constexpr (EPK) {
                                const double exm = efld(cs, 1), exq = efld(cs, 2), ea = efld(cs, 0);
                                return (ZV && k.zq) ? 0.0 : div_hh(k, stencil_sum<UN>(k, c, exq, exm, yp, ym, ea, EP));
                            } else {
                                return (ZV && k.zq) ? 0.0 : div_hh(k, stencil_sum<UN>(k, c, EXp[cs], EXm[cs], yp, ym, EA[cs], EP));
                            }
                        };
                        if constexpr (newtonish(MODE)) { // the interior rows' NEWTON expressions, exp once
                            const double we = efld(cs, 4), A = newton_A<MODE>(k, we), E = newton_E<MODE>(we);
                            const double a = newton_op(qe(), c, A, E);
                            nv = newton_update<MODE>(k, c, efld(cs, 3) - a, A, E);
                        } else {
                            const double a = op_finish<MODE>(k, qe(), c, 0.0);
                            nv = jacobi_update<MODE>(k, c, EF[cs] - a, 0.0);
                        }
                        ES1n = (!pz || !erowc) ? c : nv;
                    }
                }
                if constexpr (PRO != 0) {
                    // the corrected iterate: plane z+1 (VL) and the halo row at plane z (HL); with z0
                    // even, ph 0 has z even (z+1 odd: coarse K, K+1) and ph 1 has z odd
#pragma unroll
                    for (int j = 0; j < NV; j++)
                        correct(VL[cs][j], j, ph == 0, pok(z + 1), ph == 0 ? 0 : 1, 1, mirc);
                    correct(HL[cs], -1, ph == 1, pok(z), 0, 1, mirc);
                }
                // sweep 1 at plane z, local rows 0..RY
#pragma unroll
                for (int j = 0; j < NV; j++) {
                    const double2 c = Vc[j], zm = Vp[j], zp = VL[cs][j];
                    const double2 lm = j == 0 ? HL[cs] : Vc[j - 1], lp = j == RY ? vY : Vc[j + 1];
                    const double2 ym = M ? lp : lm, yp = M ? lm : lp;
                    double q[2];
                    if (ZV && k.zq) { // the stencil of the zero iterate over h^2: +0 exactly (Coef::zq)
                        q[0] = 0.0;
                        q[1] = 0.0;
                    } else {
                        const double xm0 = lane_from_left<true>(c.y, CL[j]);
                        const double xp1 = lane_from_right<true>(c.x, CR[j]);
                        q[0] = stencil_sum<UN>(k, c.x, c.y, xm0, yp.x, ym.x, zp.x, zm.x);
                        q[1] = stencil_sum<UN>(k, c.y, xp1, c.x, yp.y, ym.y, zp.y, zm.y);
                        div_hh_row<MODE>(k, q);
                    }
                    double a0, a1, n0, n1;
                    if constexpr (newtonish(MODE)) {
                        const double2 wv = WL[cs][j];
                        const double2 A = make_double2(newton_A<MODE>(k, wv.x), newton_A<MODE>(k, wv.y));
#ifdef GS_EXP_EFIELD
                        const double2 E = XL[cs][j];
#else
                        const double2 E = YSH ? make_double2(nb_recip(k.preFac + A.x), nb_recip(k.preFac + A.y))
                                              : make_double2(newton_E<MODE>(wv.x), newton_E<MODE>(wv.y));
#endif
                        if (!RECOMP && j >= 1) {
                            Acur[j - 1] = A;
                            Ecur[j - 1] = E;
                        }
                        if (ELDS && j >= 1) eprev_l[ph][j - 1][wx + WX * wy][lane] = E;
                        if constexpr (YSH) {
                            a0 = newton_op(q[0], c.x, A.x, 1.0);
                            a1 = newton_op(q[1], c.y, A.y, 1.0);
                            n0 = c.x + k.omega * ((FL[cs][j].x - a0) * E.x);
                            n1 = c.y + k.omega * ((FL[cs][j].y - a1) * E.y);
                        } else {
                            a0 = newton_op(q[0], c.x, A.x, E.x);
                            a1 = newton_op(q[1], c.y, A.y, E.y);
                            n0 = newton_update<MODE>(k, c.x, FL[cs][j].x - a0, A.x, E.x);
                            n1 = newton_update<MODE>(k, c.y, FL[cs][j].y - a1, A.y, E.y);
                        }
                    } else {
                        a0 = op_finish<MODE>(k, q[0], c.x, 0.0);
                        a1 = op_finish<MODE>(k, q[1], c.y, 0.0);
                        n0 = jacobi_update<MODE>(k, c.x, FL[cs][j].x - a0, 0.0);
                        n1 = jacobi_update<MODE>(k, c.y, FL[cs][j].y - a1, 0.0);
                    }
                    const double r0 = FL[cs][j].x - a0, r1 = FL[cs][j].y - a1;
                    if (partials && j >= 1 && z >= zb && z <= ze && rowc[j + 1]) {
                        if (okx0) sumsq += r0 * r0;
                        if (okx1) sumsq += r1 * r1;
                    }
                    const bool keep = !pz || !rowc[j + 1];
                    V1n[j] = make_double2((keep || bx0) ? c.x : n0, (keep || bx1) ? c.y : n1);
                }
                // sweep 2 at plane z-1, own rows 1..RY
                if (z - 1 >= zb && z - 1 <= ze) {
                    const int64_t zo = (int64_t)(z - 1) * ldz;
#pragma unroll
                    for (int j = 1; j <= RY; j++) {
                        const double2 c = V1c[j], zm = V1p[j - 1], zp = V1n[j];
                        const double2 lm = V1c[j - 1], lp = j == RY ? sY : V1c[j + 1];
                        const double2 ym = M ? lp : lm, yp = M ? lm : lp;
                        const double xm0 = lane_from_left<true>(c.y, CL[NV + j - 1]);
                        const double xp1 = lane_from_right<true>(c.x, CR[NV + j - 1]);
                        double q[2] = {stencil_sum<UN>(k, c.x, c.y, xm0, yp.x, ym.x, zp.x, zm.x),
                                       stencil_sum<UN>(k, c.y, xp1, c.x, yp.y, ym.y, zp.y, zm.y)};
                        div_hh_row<MODE>(k, q);
                        double o0, o1;
                        if constexpr (newtonish(MODE)) {
                            double2 A, E;
                            if constexpr (RECOMP) {
                                const double2 wv = wprev_l[j - 1][wx + WX * wy][lane];
                                A = make_double2(newton_A<MODE>(k, wv.x), newton_A<MODE>(k, wv.y));
                                if constexpr (ELDS) E = eprev_l[ph ^ 1][j - 1][wx + WX * wy][lane];
                                else E = make_double2(1.0, 1.0);
                            } else {
                                A = Aprev[j - 1];
                                E = Eprev[j - 1];
                            }
                            const double a0 = newton_op(q[0], c.x, A.x, YSH ? 1.0 : E.x);
                            const double a1 = newton_op(q[1], c.y, A.y, YSH ? 1.0 : E.y);
                            const double2 fp = RECOMP ? fprev_l[j - 1][wx + WX * wy][lane] : Fprev[j - 1];
                            if constexpr (YSH) {
                                o0 = c.x + k.omega * ((fp.x - a0) * E.x);
                                o1 = c.y + k.omega * ((fp.y - a1) * E.y);
                            } else {
                                o0 = newton_update<MODE>(k, c.x, fp.x - a0, A.x, E.x);
                                o1 = newton_update<MODE>(k, c.y, fp.y - a1, A.y, E.y);
                            }
                        } else {
                            const double a0 = op_finish<MODE>(k, q[0], c.x, 0.0);
                            const double a1 = op_finish<MODE>(k, q[1], c.y, 0.0);
                            o0 = jacobi_update<MODE>(k, c.x, Fprev[j - 1].x - a0, 0.0);
                            o1 = jacobi_update<MODE>(k, c.y, Fprev[j - 1].y - a1, 0.0);
                        }
                        if (yof(j) <= ny) {
                            double* qo = out + x + roff[j + 1] + zo;
                            if (okx1) st2s<NT>(qo, o0, o1);
                            else if (okx0) *qo = o0;
                        }
                    }
                }
            };
            if constexpr (!SPEC) {
                sweeps(RtBool{mir});
            } else {
                if (mir) sweeps(BoolC<true>{});
                else sweeps(BoolC<false>{});
            }
            // ---- rotate ----
#pragma unroll
            for (int j = 1; j <= RY; j++) {
                V1p[j - 1] = V1c[j];
                if (!RECOMP) Fprev[j - 1] = FL[cs][j];
                if constexpr (RECOMP) {
                    wprev_l[j - 1][wx + WX * wy][lane] = WL[cs][j];
                    fprev_l[j - 1][wx + WX * wy][lane] = FL[cs][j];
                } else if (newtonish(MODE)) {
                    Aprev[j - 1] = Acur[j - 1];
                    Eprev[j - 1] = Ecur[j - 1];
                }
            }
#pragma unroll
            for (int j = 0; j < NV; j++) {
                V1c[j] = V1n[j];
                Vp[j] = Vc[j];
                Vc[j] = VL[cs][j];
            }
            if constexpr (XH) {
                EP = EC;
                if constexpr (EPK) {
                    if (edg) EC = efld(cs, 0);
                } else {
                    EC = EA[cs];
                }
                ES1c = ES1n;
            }
            if (PRO && ph == 1) { // next step: coarse planes K+1, K+2
                if constexpr (WLDS) {
                    wsl ^= 1;
                } else {
#pragma unroll
                    for (int r = 0; r < NCR; r++) W0[r] = W1[r];
                    if constexpr (HALF) {
#pragma unroll
                        for (int r = 0; r < NCR; r++) H0[r] = H1[r];
                    }
                }
                xpass(1);
            }
        }
    }
    if (partials) {
        // fixed-order block sum: waves in (x, y) order
        sumsq = wave_sum(sumsq);
        const int wid = wx + WX * wy;
        if (lane == 0) red[wid] = sumsq;
        __syncthreads();
        if (tid == 0) {
            double t = 0.0;
            for (int i = 0; i < 2 * WX; i++) t += red[i];
            partials[tile] = t;
        }
    }
    if constexpr (TS) {
        if (tid == 0) {
            double* t = const_cast<double*>(es) + 4 * tile;
            t[0] = (double)tstart;
            t[1] = (double)wall_clock64();
            t[2] = (double)(blockIdx.x + (int64_t)gridDim.x * blockIdx.y);
            t[3] = (double)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4); // HW_ID: CU / SH / SE
        }
    }
}

// Shapes of the fused pair. Rows of <= 512 points: k_tb2y, 2 y-waves of TBY_RY rows each under the
// 4 x-waves of a row (8 waves, ~218 VGPRs: two waves per SIMD; NEWTON carries the w rows too and takes
// 2 rows per wave to stay clear of spills). Rows of <= 1024 points: k_tb2 at 2
// rows per wave in blocks of <= 8 x-waves (measured on MI355X with tools/kbench.py --pairs: at 2 rows
// a wave needs ~216 VGPRs, so two waves share a SIMD and hide each other's latency, which beats the
// lower halo overhead of 3-6 rows at one wave per SIMD by 20-25%).
constexpr int TBY_RY = 2, TBY_RY_NEWTON = 2, TBY_WX = 4, TB_RY_B = 2, TB_WX_B = 8;
// prefetch distance of k_tb2y (plane steps): LINEAR keeps two steps in flight (215 VGPRs, still two
// waves per SIMD; 0.662 vs 0.673 ms per 512^3 pair, profiles/r01m_summary.md), the other modes and
// the fused prolongation one (VGPR budget: the LINEAR prolongation pair at distance 2 spills)
constexpr int tby_pfd(int mode) { return mode == GS_LINEAR ? 2 : 1; }
// column blocks (XH): LINEAR at distance 2 too (247 VGPRs, no spill); GS_TBX_PFD=1 selects distance 1 (A/B)
bool tbx_pfd2() { return kKnobs.tbxPfd2; }

// Column blocks (k_tb2y XH) for rows of more than 512 points in LINEAR / NONLINEAR mode: 1024-point rows
// (BASELINE config #5) were k_tb2's one-y-wave shape before; GS_PAIR_XH=0 restores that (A/B).
bool xh_enabled() { return kKnobs.pairXh; }

// Geometry rule of the fused pair: the whole x-row in one block (or, XH, one column block of 512
// points) and enough work for >= 128 blocks of 4-plane chunks; the z-chunk is then chosen for >= 1024
// blocks (4..64 planes: at 512^3, 64-plane chunks measured 5-8% faster than 32 — fewer re-read
// chunk-boundary planes). Returns 0 (impossible), 1 (possible) or 2 (possible and fills the GPU);
// *y2: the k_tb2y whole-row shape, *xh: the k_tb2y column-block shape (neither: k_tb2).
// Blocks of `threads` threads kernel `fn` keeps resident on the whole GPU (occupancy x CUs, cached).
int64_t resident_blocks(const void* fn, int threads)
{
    static std::mutex m;
    static std::map<std::pair<const void*, int>, int64_t> cache;
    std::lock_guard<std::mutex> lk(m);
    const auto key = std::make_pair(fn, threads);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int per = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, threads, 0) != hipSuccess || per < 1) per = 1;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        cus = 256;
    (void)hipGetLastError();
    return cache[key] = (int64_t)per * cus;
}

// Round-aware chunking for levels whose grid is a few rounds of resident blocks: the chunk length c
// in [lo, hi] (even if `even`) maximising (blocks / (rounds x capacity)) x c / (c + halo) — whole
// rounds, long chunks (each recomputes ~halo planes) — among those that still fill the GPU.
// GS_FIT_ROUNDS=0 keeps the callers' rules (A/B). Returns 0 for "keep".
int fit_chunk(int64_t tiles, int64_t planes, int64_t cap, int lo, int hi, bool even, double halo)
{
    if (!kKnobs.fitRounds || tiles < 1 || planes < 1 || cap < 1) return 0;
    double best = -1.0;
    int bc = 0;
    for (int c = lo; c <= hi; c++) {
        if (even && (c & 1)) continue;
        const int64_t blocks = tiles * ((planes + c - 1) / c);
        if (blocks < cap && bc != 0) continue; // would leave CUs idle where a shorter chunk does not
        const int64_t rounds = (blocks + cap - 1) / cap;
        const double score = (double)blocks / (double)(rounds * cap) * c / (c + halo);
        if (score > best) {
            best = score;
            bc = c;
        }
    }
    return bc;
}

// refit a plan's z-chunk (grid.y) for kernel `fn` at `threads` threads
template <class K>
void refit_chunks(K* fn, int threads, int64_t planes, int lo, int hi, bool even, double halo, int* zc, dim3* g)
{
    const int c = fit_chunk(g->x, planes, resident_blocks((const void*)fn, threads), lo, hi, even, halo);
    if (c > 0) {
        *zc = c;
        g->y = (unsigned)((planes + c - 1) / c);
    }
}

// compute units of the current device (cached per device)
int64_t device_cus()
{
    static std::mutex m;
    static std::map<int, int64_t> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    std::lock_guard<std::mutex> lk(m);
    auto it = cache.find(dev);
    if (it != cache.end()) return it->second;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    (void)hipGetLastError();
    return cache[dev] = cus;
}

// chunk length (planes) of pair launches over plane ranges past a slab's first plane; 0: the rules
// for whole levels (A/B: GS_SLAB_ZC)
int slab_zc() { return kKnobs.slabZc; }

// the same for plane ranges from a level's first plane (whole single-GPU levels of >= 2^26 points); A/B
int whole_zc() { return kKnobs.pairZc; }

int tb2_plan(const gs_stencil* S, const gs_level* L, int* zc, dim3* grid, dim3* block, bool* y2 = nullptr,
             int mode = GS_LINEAR, bool* xh = nullptr, bool pro = false)
{
    if (!S || !L || !canonical_order(S) || L->nx < 1 || L->ny < 1 || L->nz < 1) return 0;
    const bool two = L->nx <= 2 * WAVE * TBY_WX;
    // NEWTON: column blocks from 513 points too since r04 (sweep 2's rows in LDS, edge values loaded per
    // step: 255 VGPRs, no spill): 1023^3 pair 8.83 vs 29.9 ms for k_tb2, Newton iteration 109-110 vs
    // 166-167 ms (profiles/r04/r04i_newton_1023.txt); GS_NEWTON_XH=0 keeps k_tb2 for the plain pairs (A/B).
    // NEWTON prolongation pairs (pro) have no k_tb2 form
    const bool colb = !two && xh_enabled() && L->nx <= (int64_t)1 << 20 &&
                      (!newtonish(mode) || pro || kKnobs.newtonXh || L->nx > 2 * WAVE * TB_WX_B);
    if (!two && !colb && L->nx > 2 * WAVE * TB_WX_B) return 0;
    const int64_t nh = colb ? (L->nx + 2 * WAVE * TBY_WX - 1) / (2 * WAVE * TBY_WX) : 1;
    const int rows = (two || colb) ? 2 * (newtonish(mode) ? TBY_RY_NEWTON : TBY_RY) : TB_RY_B; // output rows per block
    const int64_t tiles = (L->ny + rows - 1) / rows * nh;
    // the block count (of 4-plane chunks) from which the pair is the level's smoother: 128 takes 64^3
    // (256 blocks: ZV pair + prolongation pair 23.5 us vs 4 one-point sweeps + prolongation 24.7 us) and
    // leaves 32^3 (64 blocks: 25.2 vs 23.9 us) to the one-point kernel (rocprofv3 V-cycle traces, r02:
    // tools/rr_ab_session.sh pmb GS_PAIR_MIN_BLOCKS 512 128);
    // GS_PAIR_MIN_BLOCKS overrides it (A/B)
    const int64_t minBlocks = kKnobs.pairMinBlocks;
    const int fills = tiles * ((L->nz + 3) / 4) >= minBlocks ? 2 : 1;
    int64_t c = tiles * L->nz / 1024;
    c = c < 4 ? 4 : (c > 64 ? 64 : c);
    // levels of >= 2^26 points: chunks for ~512 blocks, up to 128 planes (one 8-wave block per CU, two
    // rounds at 512^3; fewer re-read chunk-boundary planes): 0.658 vs 0.674 ms per 512^3 pair
    // (tools/kbench.py --pairs --zc 64,96,128). GS_PAIR_BIG_CHUNKS=0 keeps the 64-plane rule (A/B).
    const bool big_chunks = kKnobs.bigChunks;
    // (k_tb2, 1024-point rows: 5.99 vs 6.12 ms per 1024^3 pair, 0.774 vs 0.779 ms on a 1024x1024x128 slab)
    if (big_chunks && L->nx * L->ny * L->nz >= ((int64_t)1 << 26)) {
        const int64_t b = tiles * L->nz / 512;
        c = b < 64 ? 64 : (b > 128 ? 128 : b);
        // k_tb2y shapes whose tiles fit the CUs: chunks long enough for ONE round of blocks (every
        // k_tb2y variant at this size runs one 8-wave block per CU). 512^3: 256 blocks of 256 planes,
        // pair 0.587 vs 0.602 ms, V-cycle 2.16 vs 2.18 ms (tools/ab_multi.sh; 170- and 192-plane
        // chunks, i.e. uneven rounds, are far slower). Only for plane ranges from the level's first plane
        // (z0 = 0: whole single-GPU levels): the interior launch of an overlapped Z-slab sweep keeps two
        // rounds, so that the ghost exchange running beside it (RCCL kernels on the comm stream) finds
        // free CUs halfway through instead of waiting for every block of the interior to retire.
        // GS_PAIR_ONE_ROUND=0 keeps the rule above (A/B).
        const bool one_round = kKnobs.oneRound;
        const int64_t cus = device_cus();
        if (one_round && (two || colb) && tiles <= cus && L->z0 == 0) {
            const int64_t per = cus / tiles; // chunks per tile
            int64_t c1 = (L->nz + per - 1) / per;
            c1 += c1 & 1;
            if (c1 > c) c = c1;
        } else if (one_round && colb && tiles > cus && L->z0 == 0) {
            // more tiles than CUs (1024^3: 512 column-block tiles): chunks for four rounds of blocks where
            // that lengthens them (1024^3: 512 planes, pair 4.90 vs 5.00-5.06 ms, tools/zc_sweep.sh,
            // profiles/r02k; a 1024x1024x128 slab keeps its 128-plane chunks, 0.622 vs 0.641 ms at 64)
            const int64_t per = std::max<int64_t>(1, 4 * cus / tiles);
            int64_t c1 = (L->nz + per - 1) / per;
            c1 += c1 & 1;
            if (c1 > c) c = c1;
        }
        // plane ranges past a slab's first plane (the interior launch of an overlapped Z-slab sweep):
        // GS_SLAB_ZC-plane chunks, so that blocks retire often and the ghost exchange's kernels
        // (RCCL's need a whole SIMD's registers) find a free CU soon after they are enqueued
        if (L->z0 != 0) {
            const int sz = slab_zc();
            if (sz > 0) c = std::max(2, sz); // >= 2: the even rounding below must not reach 0
        } else {
            const int wz = whole_zc();
            if (wz > 0) c = std::max(2, wz);
        }
    }
    if (kKnobs.midZc > 0 && L->z0 == 0 && L->nx * L->ny * L->nz < ((int64_t)1 << 26)) c = std::max(2, kKnobs.midZc);
    // GS_PAIR_ONE_ROUND_MID=1: LINEAR levels of 2^24 .. 2^26 points (256^3) in one round of blocks too (A/B)
    if (kKnobs.oneRoundMid && mode == GS_LINEAR && (two || colb) && L->z0 == 0 &&
        L->nx * L->ny * L->nz >= ((int64_t)1 << 24) && L->nx * L->ny * L->nz < ((int64_t)1 << 26)) {
        const int64_t cus = device_cus();
        if (tiles <= cus) {
            const int64_t per = cus / tiles;
            int64_t c1 = (L->nz + per - 1) / per;
            c1 += c1 & 1;
            if (c1 > c) c = c1;
        }
    }
    c &= ~(int64_t)1; // even: every chunk starts on an odd plane (the fused prolongation's parities)
    *zc = (int)c;
    *grid = dim3((unsigned)tiles, (unsigned)((L->nz + c - 1) / c));
    *block = dim3(WAVE, colb ? (unsigned)TBY_WX : (unsigned)((L->nx + 2 * WAVE - 1) / (2 * WAVE)), (two || colb) ? 2 : 1);
    if (y2) *y2 = two;
    if (xh) *xh = colb;
    return fills;
}

// Production shape of the register-blocked kernel (chosen by tools/kbench.py on MI355X,
// profiles/r01a_kbench.json): 8 rows x 128 columns per wave, 2 waves per block, non-temporal f /
// output streams. The z-chunk is chosen per launch so the grid keeps >= 2048 blocks (at most 32
// planes, at least 4); a level too small for that many 4-plane chunks runs the one-point-per-thread
// kernel instead (coarse levels are latency-bound: parallelism beats register blocking there).
constexpr int RB_RY = 2, RB_W = 4, RB_ZCMAX = 32, RB_ZCMIN = 4;
constexpr bool RB_NT = true;

struct PassPlan {
    bool rb;
    int zc;
    dim3 grid;
};

PassPlan pass_plan(const gs_stencil* S, const gs_level* L)
{
    PassPlan p{false, 0, dim3(1)};
    if (!canonical_order(S)) {
        p.grid = gn_grid(L);
        return p;
    }
    const int64_t tiles = ((L->nx + 2 * WAVE - 1) / (2 * WAVE)) * ((L->ny + RB_RY * RB_W - 1) / (RB_RY * RB_W));
    if (tiles * ((L->nz + RB_ZCMIN - 1) / RB_ZCMIN) < 1024) {
        p.grid = gn_grid(L);
        return p;
    }
    int64_t zc = L->nz * tiles / 2048;
    zc = zc < RB_ZCMIN ? RB_ZCMIN : (zc > RB_ZCMAX ? RB_ZCMAX : zc);
    if (kKnobs.rbZc > 0) zc = kKnobs.rbZc + (kKnobs.rbZc & 1); // (A/B; even: the fused restriction's plane parity)
    p.rb = true;
    p.zc = (int)zc;
    p.grid = rb_grid(L, RB_RY, RB_W, p.zc);
    return p;
}

template <int KIND, bool ADD>
int launch_pass(const gs_stencil* S, const gs_level* L, int mode, double omega, double gamma, const double* v,
                const double* f, const double* w, double* out, double* partials, hipStream_t st)
{
    // v == NULL: the zero iterate (sweeps only, not in NONLINEAR mode, whose coarse iterates are
    // restrictions, never zero)
    mode = base_mode(mode); // (GS_NEWTON_G: the one-point passes read the factor field, which holds gamma)
    if (!S || bad_level(L) || !valid_stencil(S) || (!v && (KIND != 0 || mode == GS_NONLINEAR))) return GS_EINVAL;
    if (mode < GS_LINEAR || mode > GS_NEWTON_B || (KIND == 2 && mode != GS_NONLINEAR)) return GS_EINVAL;
    if (L->nx == 0 || L->ny == 0 || L->nz == 0) return 0;
    const Coef k = make_coef(S, L, omega, gamma);
    const int nx = (int)L->nx, ny = (int)L->ny, nz = (int)L->nz;
    const PassPlan plan = pass_plan(S, L);
    if (plan.rb) {
        const dim3 g = plan.grid, b(WAVE, RB_W);
#define GS_RBU(M, Z, U) hipLaunchKernelGGL((k_rb<M, KIND, ADD, RB_RY, RB_W, true, RB_NT, false, false, Z, U>), g, b, 0, st, k, v, f, w, out, partials, nx, ny, nz, L->ldy, L->ldz, plan.zc)
#define GS_RB(M, Z) do { if (k.unit) GS_RBU(M, Z, true); else GS_RBU(M, Z, false); } while (0)
        if (!v) {
            if constexpr (KIND == 0 && !ADD) {
                if (mode == GS_LINEAR) GS_RB(GS_LINEAR, true);
                else if (mode == GS_NEWTON_B) GS_RB(GS_NEWTON_B, true);
                else GS_RB(GS_NEWTON, true);
            }
        } else if constexpr (KIND == 2) {
            GS_RB(GS_NONLINEAR, false); // the FAS operator (NONLINEAR only)
        } else if (mode == GS_LINEAR) GS_RB(GS_LINEAR, false);
        else if (mode == GS_NONLINEAR) GS_RB(GS_NONLINEAR, false);
        else if (mode == GS_NEWTON_B) GS_RB(GS_NEWTON_B, false);
        else GS_RB(GS_NEWTON, false);
#undef GS_RB
#undef GS_RBU
    } else {
        const dim3 g = plan.grid, b(GN_BX, GN_BY);
#define GS_GN(M) hipLaunchKernelGGL((k_generic<M, KIND, ADD>), g, b, 0, st, k, v, f, w, out, partials, nx, ny, nz, L->ldy, L->ldz)
        if constexpr (KIND == 2) GS_GN(GS_NONLINEAR);
        else if (mode == GS_LINEAR) GS_GN(GS_LINEAR);
        else if (mode == GS_NONLINEAR) GS_GN(GS_NONLINEAR);
        else if (mode == GS_NEWTON_B) GS_GN(GS_NEWTON_B);
        else GS_GN(GS_NEWTON);
#undef GS_GN
    }
    return launch_status();
}

} // namespace
