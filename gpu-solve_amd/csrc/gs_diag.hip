// gs_diag.hip — libgpusolve_diag.so (include/gpusolve_diag.h): measurement and tuning code that is NOT
// part of the product: the tuning variants of the sweep and pair kernels (tools/kbench.py), streaming
// bandwidth probes (bench.py's measured ceiling, tools/), the exact-division check, and k_prr — the
// pre-smoothing pair + residual + restriction in one pass, built, bit-identical and measured slower than
// the two passes the driver runs, kept as a tested operator. Only tools/, tests/ and
// bench.py's measured-ceiling leg load this library.
#include "gs_device.hpp"
#include "gpusolve_diag.h"

namespace {

// ---------------------------------------------------------------------------------------------
// The first pre-smoothing pair, the residual of its result and the full-weighting restriction in ONE
// pass (k_prr, LINEAR; CpuSolver.cpp:94-99 with preSmoothing = 2: jacobi x2, compResidual, restrict).
// Level 0 of a 2+2 V-cycle is then two passes instead of three: this kernel reads v and f once and
// writes v'' and the coarse f (25 B per fine point instead of 24 + 17).
// A block is the whole x-row — PRR_WX waves, ONE column per lane, so a lane's z-windows of four stages
// fit its registers — times a tile of PRR_T = 4 output rows y0..y0+3 (y0 odd: the tile holds the
// centres of coarse rows (y0+1)/2 and (y0+3)/2). The restriction needs r on rows y0..y0+4, r needs v''
// on y0-1..y0+5, v'' needs sweep 1 on y0-2..y0+6 and sweep 1 needs v on y0-3..y0+7: every stage's
// extra rows are recomputed in-lane (no y exchange). Wavefront along z, at step z: sweep 1 at plane
// z, sweep 2 at z-1, r at z-2, and the restriction of coarse plane Z = (z-4)/2 from r at z-5..z-3
// (one step late, so that every x-edge it reads was published before this step's one barrier).
// x-neighbours: DPP lane shifts, the columns beyond a wave's edges (v, sweep 1, sweep 2) through LDS;
// r goes to an LDS ring of five planes that the restriction reads directly. A block walks a chunk of
// coarse planes Zb..Ze: fine output planes 2Zb-1..2Ze (the last chunk up to nz), with the pipeline's
// z-halo (sweep 1 from 2Zb-3, r up to 2Ze+1) recomputed at the chunk ends. Every point uses the
// expression of k_tb2y / k_rr2 (same order, same boundary values), so v'' and the coarse f are
// bit-identical to gs_jacobi_sweep2 + gs_residual_restrict; the norm partials are those of r = f - A v
// (the input), as the speculative pair's, in this kernel's block order.
// MEASURED SLOWER than the two passes it replaces, so the driver does not use it: 1.45 vs 1.10 ms at
// 512^3 (tools/prr_bench.py). Its traffic is 1.06 x the 25 B/point, but the in-lane recomputation
// costs 21 stencil evaluations per 4 outputs against 15 for pair + k_rr2, and one column per lane
// doubles the DPP shifts: PMC 1.54 x the VALU instructions of the two kernels at 254 VGPRs (no
// prefetch room beyond one plane of v). Kept as a tested operator (tests/test_gpu_pair_restrict.py).
// ZV (r04, gs_smooth2_restrict_zero): a coarse level's first step from v = 0, whose first sweep is pointwise in f
// (q = +0): no v loads and no sweep-1 stencils, one pass over f instead of the zero-iterate pair + k_rr2 (17
// instead of 33 B per point). Measured no faster: 122 vs 62 + 63 us at a 256^3 level, 38 vs 15 + 13 us at 128^3
// (r04r, profiles/r04/r04r_zero_pair_restrict_ab.txt) — the in-lane recomputation is what costs, as at level 0.
constexpr int PRR_WX = 8, PRR_T = 4, PRR_RS = 5; // x-waves, output rows per block, r ring planes

// WXP: x-waves the block is sized for (the r ring's LDS): 8 for rows of 257-512 points, 4 / 2 for shorter rows,
// so that a 256-point level holds two blocks per CU instead of one
template <bool UN, bool ZV = false, int WXP = PRR_WX>
__global__ __launch_bounds__(WAVE* WXP) void k_prr(Coef k, const double* __restrict__ v, const double* __restrict__ f,
                                                      double* __restrict__ out, double* __restrict__ partials,
                                                      double* __restrict__ ca, double* __restrict__ cb, int nx, int ny,
                                                      int nz, int64_t ldy, int64_t ldz, int cnx, int cny, int cnz,
                                                      int64_t cldy, int64_t cldz, int ZC)
{
    // local rows i (global y0 + i): v -3..7, sweep 1 -2..6, sweep 2 -1..5, r 0..4
    constexpr int NV = 11, N1 = 9, N2 = 7, NR = 5;
    constexpr int NE = N1 + N2 + NR; // x-edge values per wave side and plane parity
    constexpr int RW = WAVE * WXP + 2; // r ring row: columns 0 .. 64 WX + 1
    __shared__ double edge[2][WXP + 2][2][NE];
    // r of the last planes, every column of the tile's rows 0..4: slot p mod 5 (the restriction at step z
    // reads planes z-5..z-3 while a wave one step ahead writes z-1 — five slots keep them apart)
    __shared__ double rring[PRR_RS][NR][RW];
    __shared__ double red[WXP];
    const int lane = threadIdx.x;
    const int wx = __builtin_amdgcn_readfirstlane(threadIdx.y);
    const int WX = blockDim.y;
    const int tid = lane + WAVE * wx;
    for (int i = tid; i < 2 * (WXP + 2) * 2 * NE; i += WAVE * WX) (&edge[0][0][0][0])[i] = 0.0;
    for (int i = tid; i < PRR_RS * NR * RW; i += WAVE * WX) (&rring[0][0][0])[i] = 0.0;
    __syncthreads();
    const int64_t tile = xcd_tile(blockIdx.x + (int64_t)gridDim.x * blockIdx.y, (int64_t)gridDim.x * gridDim.y);
    const int y0 = 1 + (int)(tile % gridDim.x) * PRR_T;
    const int Zb = 1 + (int)(tile / gridDim.x) * ZC, Ze = min(Zb + ZC - 1, cnz);
    const int zb = 2 * Zb - 1, ze = Ze == cnz ? nz : 2 * Ze; // output planes of v''
    const int rlast = 2 * Ze + 1;                            // last plane of r
    const int s2last = max(ze, rlast + 1), s1last = s2last + 1;
    const int x = 1 + wx * WAVE + lane;
    const int xl = min(x, nx + 1);
    const bool okx = x <= nx;
    int64_t roff[NV]; // rows -3..7 at index i + 3
    bool rowc[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) {
        const int y = y0 - 3 + i;
        roff[i] = (int64_t)min(max(y, 0), ny + 1) * ldy;
        rowc[i] = y >= 1 && y <= ny;
    }
    auto at = [&](const double* b, int i, int p) {
        return b + xl + roff[i + 3] + (int64_t)min(max(p, 0), nz + 1) * ldz;
    };
    auto pin = [&](int p) { return p >= 1 && p <= nz; };
    auto rslot = [](int p) { return ((p % PRR_RS) + PRR_RS) % PRR_RS; };

    double Vm[N1], Vc[NV], Vn[NV], VL[NV]; // v at z-1 (rows -2..6), z, z+1, z+2 in flight (rows -3..7)
    double F0[N1], F1[N2], F2[NR];        // f at z (rows -2..6), z-1 (-1..5), z-2 (0..4)
    double S1a[N2], S1b[N1];              // sweep 1 at z-2 (rows -1..5), z-1 (-2..6)
    double S2a[NR], S2b[N2];              // sweep 2 at z-3 (rows 0..4), z-2 (-1..5)
#pragma unroll
    for (int i = 0; i < N1; i++) Vm[i] = ZV ? 0.0 : *at(v, i - 2, zb - 3);
#pragma unroll
    for (int i = 0; i < NV; i++) {
        Vc[i] = ZV ? 0.0 : *at(v, i - 3, zb - 2);
        Vn[i] = ZV ? 0.0 : *at(v, i - 3, zb - 1);
    }
#pragma unroll
    for (int i = 0; i < N2; i++) {
        F1[i] = 0.0;
        S1a[i] = 0.0;
        S2b[i] = 0.0;
    }
#pragma unroll
    for (int i = 0; i < N1; i++) S1b[i] = 0.0;
#pragma unroll
    for (int i = 0; i < NR; i++) {
        F2[i] = 0.0;
        S2a[i] = 0.0;
    }
    double sumsq = 0.0;
    auto lds_barrier = [] {
        __builtin_amdgcn_s_waitcnt(0xc07f); // lgkmcnt(0): LDS only, the loads stay in flight
        __builtin_amdgcn_s_barrier();
    };

    for (int z = zb - 2; z <= s1last + 1; z++) {
        // ---- loads: v(z+2) for the next step, f(z) for this step's sweep 1 ----
#pragma unroll
        for (int i = 0; i < NV; i++) VL[i] = ZV ? 0.0 : *at(v, i - 3, z + 2);
#pragma unroll
        for (int i = 0; i < N1; i++) F0[i] = *at(f, i - 2, z);
        // ---- publish x-edges: v(z) rows -2..6, sweep 1 (z-1) rows -1..5, sweep 2 (z-2) rows 0..4 ----
        const int ph = z & 1;
        if (lane == 0 || lane == WAVE - 1) {
            const int sd = lane == 0 ? 0 : 1;
#pragma unroll
            for (int i = 0; i < N1; i++) edge[ph][wx + 1][sd][i] = Vc[i + 1];
#pragma unroll
            for (int i = 0; i < N2; i++) edge[ph][wx + 1][sd][N1 + i] = S1b[i + 1];
#pragma unroll
            for (int i = 0; i < NR; i++) edge[ph][wx + 1][sd][N1 + N2 + i] = S2b[i + 1];
        }
        lds_barrier();
        // the columns left of lane 0 / right of lane 63 (LDS broadcast reads, straight into the DPP's old operand)
        auto CL = [&](int i) { return edge[ph][wx][1][i]; };
        auto CR = [&](int i) { return edge[ph][wx + 2][0][i]; };

        // ---- restriction of coarse plane Z from r at 2Z-1, 2Z, 2Z+1 (= z-5, z-4, z-3), read from the ring ----
        if (!(z & 1) && (z - 4) / 2 >= Zb && (z - 4) / 2 <= Ze) {
            const int Z = (z - 4) / 2;
            const int X = x >> 1;
            const int sl[3] = {rslot(z - 5), rslot(z - 4), rslot(z - 3)};
            if (!(x & 1) && X <= cnx) {
#pragma unroll
                for (int t = 0; t < 2; t++) {
                    const int Y = (y0 + 1) / 2 + t, ic = 1 + 2 * t; // centre row y0 + ic = 2Y
                    if (Y > cny) continue;
                    double acc = 0.0;
#pragma unroll
                    for (int a = -1; a <= 1; a++)
#pragma unroll
                        for (int b = -1; b <= 1; b++)
#pragma unroll
                            for (int c = -1; c <= 1; c++) {
                                const double wgt = 0.125 * ((2.0 - (a < 0 ? -a : a)) / 2.0) *
                                                   ((2.0 - (b < 0 ? -b : b)) / 2.0) * ((2.0 - (c < 0 ? -c : c)) / 2.0);
                                acc += wgt * rring[sl[c + 1]][ic + b][x + a];
                            }
                    const int64_t q = X + Y * cldy + (int64_t)Z * cldz;
                    ca[q] = acc;
                    if (cb) cb[q] = acc;
                }
            }
        }

        // ---- sweep 1 at plane z, rows -2..6 ----
        double S1n[N1];
        if (z <= s1last) {
            double q[N1];
            if constexpr (ZV) { // v = 0: the stencil over h^2 is +0 exactly (Coef::zq, checked by the launcher)
#pragma unroll
                for (int i = 0; i < N1; i++) q[i] = 0.0;
            } else {
#pragma unroll
                for (int i = 0; i < N1; i++) {
                    const double c = Vc[i + 1];
                    const double xm = lane_from_left<true>(c, CL(i)), xp = lane_from_right<true>(c, CR(i));
                    q[i] = stencil_sum<UN>(k, c, xp, xm, Vc[i + 2], Vc[i], Vn[i + 1], Vm[i]);
                }
                div_hh_n(k, q);
            }
            const bool pz = pin(z);
            const bool own = partials && z >= zb && z <= ze && pz && okx;
#pragma unroll
            for (int i = 0; i < N1; i++) {
                const double c = Vc[i + 1];
                const double r0 = F0[i] - q[i];
                const double n = jacobi_update<GS_LINEAR>(k, c, r0, 0.0);
                S1n[i] = (pz && rowc[i + 1] && okx) ? n : c;
                if (own && i >= 2 && i <= 5 && rowc[i + 1]) sumsq += r0 * r0;
            }
        } else {
#pragma unroll
            for (int i = 0; i < N1; i++) S1n[i] = 0.0;
        }
        // ---- sweep 2 at plane z-1, rows -1..5 (stored: rows 0..3 of the output planes) ----
        double S2n[N2];
        if (z - 1 >= zb - 1 && z - 1 <= s2last) {
            double q[N2];
#pragma unroll
            for (int i = 0; i < N2; i++) {
                const double c = S1b[i + 1];
                const double xm = lane_from_left<true>(c, CL(N1 + i)), xp = lane_from_right<true>(c, CR(N1 + i));
                q[i] = stencil_sum<UN>(k, c, xp, xm, S1b[i + 2], S1b[i], S1n[i + 1], S1a[i]);
            }
            div_hh_n(k, q);
            const int p = z - 1;
            const bool pz = pin(p);
            const bool st = p >= zb && p <= ze && pz && okx;
#pragma unroll
            for (int i = 0; i < N2; i++) {
                const double c = S1b[i + 1];
                const double n = jacobi_update<GS_LINEAR>(k, c, F1[i] - q[i], 0.0);
                S2n[i] = (pz && rowc[i + 2] && okx) ? n : c;
                if (st && i >= 1 && i <= 4 && rowc[i + 2])
                    __builtin_nontemporal_store(n, out + x + roff[i + 2] + (int64_t)p * ldz);
            }
        } else {
#pragma unroll
            for (int i = 0; i < N2; i++) S2n[i] = 0.0;
        }
        // ---- r = f - A v'' at plane z-2, rows 0..4 (0 outside the interior) -> the ring ----
        if (z - 2 >= zb && z - 2 <= rlast) {
            double q[NR];
#pragma unroll
            for (int i = 0; i < NR; i++) {
                const double c = S2b[i + 1];
                const double xm = lane_from_left<true>(c, CL(N1 + N2 + i)), xp = lane_from_right<true>(c, CR(N1 + N2 + i));
                q[i] = stencil_sum<UN>(k, c, xp, xm, S2b[i + 2], S2b[i], S2n[i + 1], S2a[i]);
            }
            div_hh_n(k, q);
            const bool pz = pin(z - 2);
            const int sl = rslot(z - 2);
#pragma unroll
            for (int i = 0; i < NR; i++) rring[sl][i][x] = (pz && rowc[i + 3] && okx) ? F2[i] - q[i] : 0.0;
        }
        // ---- rotate ----
#pragma unroll
        for (int i = 0; i < NR; i++) {
            S2a[i] = S2b[i + 1];
            F2[i] = F1[i + 1];
        }
#pragma unroll
        for (int i = 0; i < N2; i++) {
            S2b[i] = S2n[i];
            S1a[i] = S1b[i + 1];
            F1[i] = F0[i + 1];
        }
#pragma unroll
        for (int i = 0; i < N1; i++) {
            S1b[i] = S1n[i];
            Vm[i] = Vc[i + 1];
        }
#pragma unroll
        for (int i = 0; i < NV; i++) {
            Vc[i] = Vn[i];
            Vn[i] = VL[i];
        }
    }
    if (partials) {
        sumsq = wave_sum(sumsq);
        if (lane == 0) red[wx] = sumsq;
        __syncthreads();
        if (tid == 0) {
            double t = 0.0;
            for (int i = 0; i < WX; i++) t += red[i];
            partials[tile] = t;
        }
    }
}

// k_prr geometry: the whole row in one block (<= 512 points), 4-row tiles, chunks of coarse planes for
// ~512 blocks (one 8-wave block per CU, two rounds at 512^3; 4..64 coarse planes: the chunk ends
// recompute five planes of the pipeline)
static bool prr_plan(const gs_stencil* S, const gs_level* fl, const gs_level* cl, int mode, int* zc, dim3* g, dim3* b)
{
    if (!S || !valid_stencil(S) || !canonical_order(S) || mode != GS_LINEAR || bad_level(fl) || bad_level(cl) ||
        !make_coef(S, fl, 0.0, 0.0).unit || // the unit-neighbour stencil sum (the general one spills here)
        fl->z0 != 0 || cl->z0 != 0 || fl->nx < 1 || fl->nx > WAVE * PRR_WX || fl->ny < 1 || fl->nz < 2 ||
        cl->nx != fl->nx / 2 || cl->ny != fl->ny / 2 || cl->nz != fl->nz / 2 || cl->nx < 1 || cl->ny < 1)
        return false;
    const int64_t tiles = (fl->ny + PRR_T - 1) / PRR_T;
    int64_t c = (cl->nz * tiles + 511) / 512;
    c = c < 4 ? 4 : (c > 64 ? 64 : c);
    *zc = (int)c;
    *g = dim3((unsigned)tiles, (unsigned)((cl->nz + c - 1) / c));
    *b = dim3(WAVE, (unsigned)((fl->nx + WAVE - 1) / WAVE));
    return true;
}


// ---- tuning variants of the LINEAR sweep (tools/kbench.py) -------------------------------------
using RbKernel = void (*)(Coef, const double*, const double*, const double*, double*, double*, int, int, int, int64_t,
                          int64_t, int);
struct Variant {
    const char* name;
    int ry, wy, zc;
    bool oneD;
    RbKernel kern;
};
#define GS_VX(RY, W, ZC, NT, X, NTV, TAG) \
    {"rb ry" #RY " w" #W " zc" #ZC " " TAG, RY, W, ZC, X, k_rb<GS_LINEAR, 0, false, RY, W, true, NT, X, NTV>}
const Variant kVariants[] = {
    GS_VX(2, 4, 32, true, false, false, "dpp nt (production shape)"),
    GS_VX(2, 4, 32, false, false, false, "dpp"),
    GS_VX(2, 4, 32, true, true, false, "dpp nt xcd"),
    GS_VX(2, 4, 32, true, false, true, "dpp nt ntv"),
    GS_VX(2, 4, 16, true, false, false, "dpp nt"),
    GS_VX(2, 4, 64, true, false, false, "dpp nt"),
    GS_VX(2, 8, 32, true, false, false, "dpp nt"),
    GS_VX(2, 2, 32, true, false, false, "dpp nt"),
    GS_VX(1, 8, 32, true, false, false, "dpp nt"),
    GS_VX(4, 4, 32, true, false, false, "dpp nt"),
    GS_VX(4, 2, 32, true, false, false, "dpp nt"),
    GS_VX(8, 2, 32, true, false, false, "dpp nt"),
};
#undef GS_VX
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

// Bandwidth ceilings. KIND 0 read a, 1 write out, 2 copy a->out, 3 triad out = a + 0.8 b.
// UNROLL independent dwordx4 per thread per iteration, NT non-temporal loads/stores.
template <int KIND, int UNROLL, bool NT>
__global__ __launch_bounds__(256) void k_bw(double* __restrict__ out, const double* __restrict__ a,
                                            const double* __restrict__ b, int64_t n2, double* __restrict__ sink)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    double acc = 0.0;
    for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i0 < n2; i0 += stride * UNROLL) {
        double2 va[UNROLL], vb[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) {
            const int64_t i = i0 + u * stride;
            if (i < n2) {
                if (KIND != 1) va[u] = ld2s<NT>(a + 2 * i);
                if (KIND == 3) vb[u] = ld2s<NT>(b + 2 * i);
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; u++) {
            const int64_t i = i0 + u * stride;
            if (i >= n2) continue;
            if (KIND == 0) acc += va[u].x + va[u].y;
            else if (KIND == 1) st2s<NT>(out + 2 * i, 1.0, 2.0);
            else if (KIND == 2) st2s<NT>(out + 2 * i, va[u].x, va[u].y);
            else st2s<NT>(out + 2 * i, va[u].x + 0.8 * vb[u].x, va[u].y + 0.8 * vb[u].y);
        }
    }
    if (KIND == 0 && acc == -1.2345e300) *sink = acc; // keeps the loads alive
}

// The same streams in the guide's shape (MI355X_MICROARCH.md: "6.29 TB/s measured, float4 copy"): no grid-stride
// loop, a grid that covers the array once, each thread UNROLL dwordx4 at stride 256 inside its block's contiguous
// run of UNROLL x 4 KB (every wave-instruction 1 KB contiguous); KIND as k_bw.
template <int KIND, int UNROLL, bool NT>
__global__ __launch_bounds__(256) void k_bwflat(double* __restrict__ out, const double* __restrict__ a,
                                                const double* __restrict__ b, int64_t n2, double* __restrict__ sink)
{
    const int64_t i0 = (int64_t)blockIdx.x * (256 * UNROLL) + threadIdx.x;
    double2 va[UNROLL], vb[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
        const int64_t i = i0 + 256 * u;
        if (i < n2) {
            if (KIND != 1) va[u] = ld2s<NT>(a + 2 * i);
            if (KIND == 3) vb[u] = ld2s<NT>(b + 2 * i);
        }
    }
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
        const int64_t i = i0 + 256 * u;
        if (i >= n2) continue;
        if (KIND == 0) acc += va[u].x + va[u].y;
        else if (KIND == 1) st2s<NT>(out + 2 * i, 1.0, 2.0);
        else if (KIND == 2) st2s<NT>(out + 2 * i, va[u].x, va[u].y);
        else st2s<NT>(out + 2 * i, va[u].x + 0.8 * vb[u].x, va[u].y + 0.8 * vb[u].y);
    }
    if (KIND == 0 && acc == -1.2345e300) *sink = acc; // keeps the loads alive
}

// The LINEAR pair's memory skeleton without its arithmetic (r06 probe, verdict r05 item 2: where does the pair lose
// against the flat triad?): k_tb2y's tiles (4 x-waves x 2 mirrored y-waves, RY = 2 rows per wave, one 4-row x 512-
// column tile per block, XCD-aware tile order), its z-march over chunks of ZC planes, its loads per plane step (v rows
// -1..RY, f rows 0..RY, dwordx4 per lane) with PFD steps in flight, and its stores (the wave's RY rows, one plane per
// step) — but each output is a pointwise mix of the loaded values, no stencil, no LDS. BAR: the pair's per-step
// workgroup barrier. 24 B per point like the pair.
// SYNC > 0: bounded drift — before plane step i a block's leader lane waits (bounded spin) until every block has
// finished step i - SYNC (a relaxed agent-scope counter, one add per block and step), so the blocks march the
// planes together (the concurrent address footprint stays a few planes wide)
template <int PFD, bool BAR, bool NTS, bool NTF, bool LEAN = false, int SYNC = 0, int RYT = 2>
__global__ __launch_bounds__(512) void k_march(const double* __restrict__ v, const double* __restrict__ f,
                                               double* __restrict__ out, int nx, int ny, int nz, int64_t ldy,
                                               int64_t ldz, int ZC, unsigned* __restrict__ cnt = nullptr)
{
    constexpr int RY = RYT, NV = RY + 1, NS = PFD == 2 ? 4 : 2;
    const int lane = threadIdx.x;
    const int wx = __builtin_amdgcn_readfirstlane(threadIdx.y);
    const int wy = __builtin_amdgcn_readfirstlane(threadIdx.z);
    const int64_t tile = xcd_tile(blockIdx.x + (int64_t)gridDim.x * blockIdx.y, (int64_t)gridDim.x * gridDim.y);
    const int y0 = 1 + (int)(tile % gridDim.x) * (2 * RY);
    const int zb = 1 + (int)(tile / gridDim.x) * ZC, ze = min(zb + ZC - 1, nz);
    const int x = 1 + wx * (2 * WAVE) + 2 * lane, xl = min(x, nx + 1);
    const bool okx = x + 1 <= nx;
    int64_t roff[RY + 2];
    bool rowc[RY + 2];
#pragma unroll
    for (int j = -1; j <= RY; j++) {
        const int y = wy ? y0 + 2 * RY - j : y0 - 1 + j;
        roff[j + 1] = (int64_t)min(max(y, 0), ny + 1) * ldy;
        rowc[j + 1] = y >= 1 && y <= ny;
    }
    auto at = [&](const double* b, int j, int z) { return b + xl + roff[j + 1] + (int64_t)min(z, nz + 1) * ldz; };
    double2 VL[NS][NV], FL[NS][NV], HL[NS];
    // LEAN: only the rows the wave stores (v and f rows 1..RY: 16 B per point of L2 requests, the triad's), the
    // others taken as zero
    auto load_slot = [&](int s, int z) {
#pragma unroll
        for (int j = 0; j < NV; j++) {
            VL[s][j] = (LEAN && j == 0) ? make_double2(0.0, 0.0) : ld2(at(v, j, z));
            FL[s][j] = (LEAN && j == 0) ? make_double2(0.0, 0.0) : ld2s<NTF>(at(f, j, z));
        }
        HL[s] = LEAN ? make_double2(0.0, 0.0) : ld2(at(v, -1, z));
    };
#pragma unroll
    for (int p = 0; p < PFD; p++) load_slot(p, zb + p);
    const bool leader = lane == 0 && wx == 0 && wy == 0;
    const unsigned nblk = gridDim.x * gridDim.y;
    for (int z0 = zb; z0 <= ze; z0 += NS) {
#pragma unroll
        for (int u = 0; u < NS; u++) {
            const int z = z0 + u;
            if (SYNC > 0) {
                const int i = z - zb;
                if (leader && i >= SYNC) {
                    const unsigned need = nblk * (unsigned)(i - SYNC + 1);
                    for (int spin = 0; spin < 2000; spin++) {
                        if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need) break;
                        __builtin_amdgcn_s_sleep(2);
                    }
                }
                __builtin_amdgcn_s_barrier();
            }
            load_slot((u + PFD) % NS, z + PFD);
            if (BAR) __builtin_amdgcn_s_barrier();
            if (SYNC > 0 && leader && z <= ze)
                __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (z <= ze) {
#pragma unroll
                for (int j = 1; j <= RY; j++) {
                    const double2 a = VL[u][j], b = j == 1 ? VL[u][0] : VL[u][j - 1], c = FL[u][j];
                    const double2 h = j == 1 ? HL[u] : FL[u][0];
                    const double o0 = a.x + 0.25 * b.x + 0.8 * c.x + 1e-300 * h.x;
                    const double o1 = a.y + 0.25 * b.y + 0.8 * c.y + 1e-300 * h.y;
                    if (rowc[j + 1] && okx) st2s<NTS>(out + xl + roff[j + 1] + (int64_t)z * ldz, o0, o1);
                }
            }
        }
    }
}

// One workgroup's operator-phase floor (r06, the one-launch coarse cycle's ~1 us per phase): `phases` rounds of
// [every thread: WORK (0: none, 1: 7 LDS reads + a dependent FP64 chain of ~14 ops, 2: the same from global memory
// (L2-resident) with a global store) -> store -> barrier]. threads: 512 or 1024.
template <int WORK>
__global__ __launch_bounds__(1024) void k_phase_probe(double* __restrict__ g, int phases, double* __restrict__ sink)
{
    __shared__ double a[2][1024 + 64];
    const int t = threadIdx.x;
    a[0][t] = t * 1e-3;
    a[1][t] = 0.0;
    if (t < 64) a[0][1024 + t] = a[1][1024 + t] = 0.0;
    __syncthreads();
    double acc = 0.0;
    for (int ph = 0; ph < phases; ph++) {
        const int s = ph & 1;
        double v = 0.0;
        if (WORK == 1) {
            const double* x = a[s] + t;
            double q = 6.0 * x[0] - x[1] - x[2] - x[3] - x[5] - x[9] - x[17];
            q = q * 0.37 + 1e-3;
            v = x[0] + 0.8 * (0.1 * (x[0] * 0.5 - q));
        } else if (WORK == 2) {
            const double* x = g + (s ? 4096 : 0) + t;
            double q = 6.0 * x[0] - x[1] - x[2] - x[3] - x[5] - x[9] - x[17];
            q = q * 0.37 + 1e-3;
            v = x[0] + 0.8 * (0.1 * (x[0] * 0.5 - q));
            g[(s ? 0 : 4096) + t] = v;
        }
        a[s ^ 1][t] = v;
        acc += v;
        __syncthreads();
    }
    if (acc == -1.2345e300) *sink = acc;
}

// A copy with the resource footprint of RCCL's gfx950 transport kernels (ncclDevKernel_Generic: 256
// VGPRs, 37664 B of LDS per 256-thread workgroup): the clobber of v255 makes the allocator reserve
// every VGPR. Stands in for the ghost exchange in tools/exchange_probe.py (when does a workgroup
// that needs a whole SIMD's registers get a CU while the interior pair holds the GPU?).
__global__ __launch_bounds__(256) void k_fatcopy(double* __restrict__ out, const double* __restrict__ a, int64_t n2)
{
    __shared__ double pad[4708];
    asm volatile("" ::: "v255");
    for (int i = threadIdx.x; i < 4708; i += 256) pad[i] = 0.0;
    __syncthreads();
    const double z = pad[(threadIdx.x * 17) % 4708];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n2; i += stride) {
        const double2 x = ld2s<true>(a + 2 * i);
        st2s<true>(out + 2 * i, x.x + z, x.y + z);
    }
}

// One wave that sleeps `iters` x s_sleep(127) (~3.4 us each at 2.4 GHz) and touches no memory: a delay
// on a stream, e.g. between the boundary planes and the interior launch of an overlapped Z-slab sweep
// so that the exchange's kernels are dispatched first (tools/exchange_probe.py).
__global__ __launch_bounds__(64) void k_sleep(int64_t iters)
{
    for (int64_t i = 0; i < iters; i++) __builtin_amdgcn_s_sleep(127);
}

// div_hh against the plain division (tests: bitwise equality over all magnitudes)
__global__ __launch_bounds__(256) void k_div_check(const double* __restrict__ a, int64_t n, Coef k,
                                                   double* __restrict__ fast, double* __restrict__ ref)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    fast[i] = div_hh(k, a[i]);
    ref[i] = a[i] / k.hh;
}

// GS_NEWTON_B's Jacobi quotient (nb_quot) of r[i] / den[i] (tests: ulp distance to the IEEE quotient)
__global__ __launch_bounds__(256) void k_nb_quot(const double* __restrict__ r, const double* __restrict__ den, int64_t n,
                                                 double* __restrict__ q)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) q[i] = nb_quot(r[i], den[i]);
}

__global__ __launch_bounds__(256) void k_triad(double* __restrict__ out, const double* __restrict__ a,
                                               const double* __restrict__ b, int64_t n2)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n2; i += stride) {
        const double2 x = reinterpret_cast<const double2*>(a)[i], y = reinterpret_cast<const double2*>(b)[i];
        reinterpret_cast<double2*>(out)[i] = make_double2(x.x + 0.8 * y.x, x.y + 0.8 * y.y);
    }
}

} // namespace

// =============================================================================================
extern "C" {

int gs_jacobi_sweep2_restrict_supported(const gs_stencil* S, const gs_level* fl, const gs_level* cl, int mode)
{
    int zc;
    dim3 g, b;
    return prr_plan(S, fl, cl, mode, &zc, &g, &b) ? 1 : 0;
}

int64_t gs_jacobi_sweep2_restrict_num_partials(const gs_stencil* S, const gs_level* fl, const gs_level* cl)
{
    int zc;
    dim3 g, b;
    return prr_plan(S, fl, cl, GS_LINEAR, &zc, &g, &b) ? (int64_t)g.x * g.y : 0;
}

int gs_jacobi_sweep2_restrict(const gs_stencil* S, const gs_level* fl, double omega, const double* v_in,
                              double* v_out, const double* f, double* partials, double* ca, double* cb,
                              const gs_level* cl, hipStream_t st)
{
    int zc;
    dim3 g, b;
    if (!prr_plan(S, fl, cl, GS_LINEAR, &zc, &g, &b) || !v_in || !v_out || !f || !ca || v_in == v_out)
        return GS_EINVAL;
    const Coef k = make_coef(S, fl, omega, 0.0);
    hipLaunchKernelGGL((k_prr<true>), g, b, 0, st, k, v_in, f, v_out, partials, ca, cb, (int)fl->nx, (int)fl->ny,
                       (int)fl->nz, fl->ldy, fl->ldz, (int)cl->nx, (int)cl->ny, (int)cl->nz, cl->ldy, cl->ldz, zc);
    return launch_status();
}

// a coarse level's first down-leg step from v = 0 in one pass (gs_device.hpp k_prr<UN=true, ZV=true>): the first
// sweep of a zero iterate is pointwise in f (q = +0, Coef::zq), so sweep 2, the residual and the restriction
// follow from f alone
int gs_smooth2_restrict_zero_supported(const gs_stencil* S, const gs_level* fl, const gs_level* cl, int mode)
{
    int zc;
    dim3 g, b;
    return (prr_plan(S, fl, cl, mode, &zc, &g, &b) && make_coef(S, fl, 0.0, 0.0).zq) ? 1 : 0;
}

int gs_smooth2_restrict_zero(const gs_stencil* S, const gs_level* fl, double omega, double* v_out, const double* f,
                             double* coarse_f, const gs_level* cl, hipStream_t st)
{
    int zc;
    dim3 g, b;
    if (!gs_smooth2_restrict_zero_supported(S, fl, cl, GS_LINEAR) || !v_out || !f || !coarse_f ||
        !prr_plan(S, fl, cl, GS_LINEAR, &zc, &g, &b))
        return GS_EINVAL;
    const Coef k = make_coef(S, fl, omega, 0.0);
#define GS_ZPRR(WXP) hipLaunchKernelGGL((k_prr<true, true, WXP>), g, b, 0, st, k, nullptr, f, v_out, nullptr, coarse_f, nullptr, \
                       (int)fl->nx, (int)fl->ny, (int)fl->nz, fl->ldy, fl->ldz, (int)cl->nx, (int)cl->ny, (int)cl->nz, \
                       cl->ldy, cl->ldz, zc)
    if (b.y <= 2) GS_ZPRR(2);
    else if (b.y <= 4) GS_ZPRR(4);
    else GS_ZPRR(PRR_WX);
#undef GS_ZPRR
    return launch_status();
}

int gs_debug_num_variants(void) { return kNumVariants; }

const char* gs_debug_variant_name(int variant)
{
    return (variant >= 0 && variant < kNumVariants) ? kVariants[variant].name : "";
}

int gs_debug_sweep_variant(int variant, const gs_stencil* S, const gs_level* L, double omega, const double* v_in,
                           double* v_out, const double* f, hipStream_t st)
{
    if (variant < 0 || variant >= kNumVariants || !S || bad_level(L) || !canonical_order(S) || !v_in || !v_out ||
        !f || v_in == v_out)
        return GS_EINVAL;
    if (L->nx == 0 || L->ny == 0 || L->nz == 0) return 0;
    const Variant& V = kVariants[variant];
    const Coef k = make_coef(S, L, omega, 0.0);
    hipLaunchKernelGGL(V.kern, rb_grid(L, V.ry, V.wy, V.zc, V.oneD), dim3(WAVE, V.wy), 0, st, k, v_in, f, nullptr,
                       v_out, nullptr, (int)L->nx, (int)L->ny, (int)L->nz, L->ldy, L->ldz, V.zc);
    return launch_status();
}

// Fused-pair shapes for tools/kbench.py --pairs (LINEAR): output rows per wave x max waves per
// block (the launch bound, hence the VGPR budget: 4 waves -> 512, 8 waves -> 256 per lane).
struct PairVariant {
    const char* name;
    int ry, wxmax, wy;
    void (*kern)(Coef, const double*, const double*, const double*, double*, double*, int, int, int, int64_t,
                 int64_t, int, int, int, const double*, const double*, int, int, int, int64_t, int64_t, const double*);
};
#define GS_PV(RY, WX) {"tb2 ry" #RY " wx" #WX, RY, WX, 1, k_tb2<GS_LINEAR, RY, WX, true>}
#define GS_PVF(RY, WX) {"tb2 ry" #RY " wx" #WX " f-cached", RY, WX, 1, k_tb2<GS_LINEAR, RY, WX, true, false>}
#define GS_PVY(RY, NTF, SPEC, TAG) {"tb2y ry" #RY " wx4 wy2" TAG, RY, 4, 2, k_tb2y<GS_LINEAR, RY, 4, true, NTF, false, SPEC>}
const PairVariant kPairVariants[] = {GS_PVF(2, 4),
                                     GS_PVF(2, 8),
                                     GS_PV(2, 4),
                                     GS_PVY(2, false, false, " f-cached"),
                                     GS_PVY(3, false, false, " f-cached"),
                                     GS_PVY(2, false, true, " f-cached spec"),
                                     GS_PVY(3, false, true, " f-cached spec"),
                                     GS_PVY(3, true, false, " f-nt"),
                                     {"tb2y ry2 wx4 wy2 f-cached spec pfd2", 2, 4, 2,
                                      k_tb2y<GS_LINEAR, 2, 4, true, false, false, true, 0, 2>},
                                     {"tb2y ry2 wx4 wy2 f-nt spec pfd2", 2, 4, 2,
                                      k_tb2y<GS_LINEAR, 2, 4, true, true, false, true, 0, 2>}};
#undef GS_PVY
#undef GS_PVF
#undef GS_PV
constexpr int kNumPairVariants = (int)(sizeof(kPairVariants) / sizeof(kPairVariants[0]));

int gs_debug_num_pair_variants(void) { return kNumPairVariants; }
const char* gs_debug_pair_variant_name(int variant)
{
    return (variant >= 0 && variant < kNumPairVariants) ? kPairVariants[variant].name : "";
}

int gs_debug_pair_variant(int variant, const gs_stencil* S, const gs_level* L, double omega, const double* v_in,
                          double* v_out, const double* f, int zc, hipStream_t st)
{
    if (variant < 0 || variant >= kNumPairVariants || !S || bad_level(L) || !canonical_order(S) || !v_in ||
        !v_out || !f || v_in == v_out || zc < 0)
        return GS_EINVAL;
    const PairVariant& V = kPairVariants[variant];
    const int64_t wx = (L->nx + 2 * WAVE - 1) / (2 * WAVE);
    if (L->nx < 1 || L->ny < 1 || L->nz < 1 || wx > V.wxmax) return GS_EINVAL;
    const int64_t tiles = (L->ny + V.ry * V.wy - 1) / (V.ry * V.wy);
    if (zc == 0) {
        int64_t c = tiles * L->nz / 1024;
        zc = (int)(c < 4 ? 4 : (c > 32 ? 32 : c));
    }
    const Coef k = make_coef(S, L, omega, 0.0);
    hipLaunchKernelGGL(V.kern, dim3((unsigned)tiles, (unsigned)((L->nz + zc - 1) / zc)), dim3(WAVE, (unsigned)wx, V.wy), 0,
                       st, k, v_in, f, nullptr, v_out, nullptr, (int)L->nx, (int)L->ny, (int)L->nz, L->ldy, L->ldz, zc,
                       0, 0, nullptr, nullptr, 0, 0, 0, (int64_t)0, (int64_t)0, nullptr);
    return launch_status();
}

// The production LINEAR pair (k_tb2y, PFD 2, plan of gs_jacobi_sweep2 unless zc > 0) with a per-block
// record in ts (4 doubles per block: start / end wall clock at 100 MHz, hardware block index, HW_ID):
// how evenly one round of blocks finishes (tools/pair_tail.py)
int gs_debug_pair_timestamps(const gs_stencil* S, const gs_level* L, double omega, const double* v_in, double* v_out,
                             const double* f, int zc, double* ts, hipStream_t st)
{
    int zcp;
    dim3 g, b;
    bool y2 = false, xh = false;
    if (!S || bad_level(L) || !valid_stencil(S) || !v_in || !v_out || !f || !ts || v_in == v_out || zc < 0 ||
        !tb2_plan(S, L, &zcp, &g, &b, &y2, GS_LINEAR, &xh) || !y2)
        return GS_EINVAL;
    if (zc > 0) {
        zcp = zc;
        g.y = (unsigned)((L->nz + zc - 1) / zc);
    }
    const Coef k = make_coef(S, L, omega, 0.0);
#define GS_TSP(U) hipLaunchKernelGGL((k_tb2y<GS_LINEAR, TBY_RY, TBY_WX, true, false, false, true, 0, 2, false, U, true>), g, b, 0, st, k, v_in, f, nullptr, v_out, nullptr, (int)L->nx, (int)L->ny, (int)L->nz, L->ldy, L->ldz, zcp, 0, 0, nullptr, nullptr, 0, 0, 0, (int64_t)0, (int64_t)0, ts)
    if (k.unit) GS_TSP(true);
    else GS_TSP(false);
#undef GS_TSP
    return launch_status();
}

// Timing only: the production LINEAR pair marching the planes in descending order (reverse != 0: every
// field viewed through plane nz + 1 - z, a negative plane pitch). The z-terms then enter the stencil sum
// swapped, so the values are NOT the sweep's; the launch moves the same bytes in the opposite plane
// order (tools/mall_probe.py: does a launch that starts where its predecessor ended find those planes in
// the Infinity Cache?)
int gs_debug_pair_reverse(const gs_stencil* S, const gs_level* L, double omega, const double* v_in, double* v_out,
                          const double* f, int reverse, hipStream_t st)
{
    int zc;
    dim3 g, b;
    bool y2 = false, xh = false;
    if (!S || bad_level(L) || !valid_stencil(S) || !v_in || !v_out || !f || v_in == v_out ||
        !tb2_plan(S, L, &zc, &g, &b, &y2, GS_LINEAR, &xh) || !y2)
        return GS_EINVAL;
    const Coef k = make_coef(S, L, omega, 0.0);
    const int64_t sh = (reverse & 1) ? (L->nz + 1) * L->ldz : 0, ldz = (reverse & 1) ? -L->ldz : L->ldz;
#define GS_RVP(U, NT) hipLaunchKernelGGL((k_tb2y<GS_LINEAR, TBY_RY, TBY_WX, NT, false, false, true, 0, 2, false, U>), g, b, 0, st, k, v_in + sh, f + sh, nullptr, v_out + sh, nullptr, (int)L->nx, (int)L->ny, (int)L->nz, L->ldy, ldz, zc, 0, 0, nullptr, nullptr, 0, 0, 0, (int64_t)0, (int64_t)0, nullptr)
    // reverse bit 1: ordinary (not non-temporal) stores of the output
    if (reverse & 2) {
        if (k.unit) GS_RVP(true, false);
        else GS_RVP(false, false);
    } else {
        if (k.unit) GS_RVP(true, true);
        else GS_RVP(false, true);
    }
#undef GS_RVP
    return launch_status();
}

// The LINEAR pair (k_tb2y, whole 512-point rows) in other row / prefetch / occupancy shapes (r06, verdict r05 item 2):
// ry output rows per y-wave (1 or 2), pfd plane steps of prefetch, wpe waves per SIMD the allocation must allow
// (0: one, the production build; 4: <= 128 VGPRs, so two 8-wave blocks share a CU), zc planes per chunk. Same
// expressions per point as the production pair, so the output is bit-identical to gs_jacobi_sweep2's.
int gs_debug_pair_shape(const gs_stencil* S, const gs_level* L, double omega, const double* v_in, double* v_out,
                        const double* f, int ry, int pfd, int wpe, int zc, hipStream_t st)
{
    if (!S || bad_level(L) || !valid_stencil(S) || !canonical_order(S) || !v_in || !v_out || !f || v_in == v_out ||
        zc < 2 || (zc & 1) || L->nx > 2 * WAVE * TBY_WX || (ry != 1 && ry != 2) || (pfd != 1 && pfd != 2) ||
        (wpe != 0 && wpe != 3 && wpe != 4))
        return GS_EINVAL;
    const Coef k = make_coef(S, L, omega, 0.0);
    const dim3 g((unsigned)((L->ny + 2 * ry - 1) / (2 * ry)), (unsigned)((L->nz + zc - 1) / zc)),
        b(WAVE, (unsigned)((L->nx + 2 * WAVE - 1) / (2 * WAVE)), 2);
    using K = void (*)(Coef, const double*, const double*, const double*, double*, double*, int, int, int, int64_t,
                       int64_t, int, int, int, const double*, const double*, int, int, int, int64_t, int64_t,
                       const double*);
#define GS_PSH(RY, P, W) k_tb2y<GS_LINEAR, RY, TBY_WX, true, false, false, true, 0, P, false, true, false, W>
    static const K tab[2][2][3] = {{{GS_PSH(1, 1, 0), GS_PSH(1, 1, 3), GS_PSH(1, 1, 4)},
                                    {GS_PSH(1, 2, 0), GS_PSH(1, 2, 3), GS_PSH(1, 2, 4)}},
                                   {{GS_PSH(2, 1, 0), GS_PSH(2, 1, 3), GS_PSH(2, 1, 4)},
                                    {GS_PSH(2, 2, 0), GS_PSH(2, 2, 3), GS_PSH(2, 2, 4)}}};
#undef GS_PSH
    if (!k.unit) return GS_EINVAL; // (the unit-stencil sums only: every reference config)
    hipLaunchKernelGGL(tab[ry - 1][pfd - 1][wpe == 0 ? 0 : (wpe == 3 ? 1 : 2)], g, b, 0, st, k, v_in, f, nullptr, v_out,
                       nullptr, (int)L->nx, (int)L->ny, (int)L->nz, L->ldy, L->ldz, zc, 0, 0, nullptr, nullptr, 0, 0,
                       0, (int64_t)0, (int64_t)0, nullptr);
    return launch_status();
}

int64_t gs_debug_pair_blocks(const gs_stencil* S, const gs_level* L, int zc)
{
    int zcp;
    dim3 g, b;
    if (!S || bad_level(L) || !valid_stencil(S) || !tb2_plan(S, L, &zcp, &g, &b, nullptr, GS_LINEAR)) return 0;
    if (zc > 0) g.y = (unsigned)((L->nz + zc - 1) / zc);
    return (int64_t)g.x * g.y;
}

int gs_debug_bw(int kind, int unroll, int nt, int blocks, double* out, const double* a, const double* b, int64_t n,
                double* sink, hipStream_t st)
{
    if (kind == 5) { // k_sleep: n iterations of s_sleep(127), one wave
        if (n < 0) return GS_EINVAL;
        hipLaunchKernelGGL(k_sleep, dim3(1), dim3(64), 0, st, n);
        return launch_status();
    }
    if (n < 0 || (n & 1) || kind < 0 || kind > 4 || (kind == 4 && blocks <= 0)) return GS_EINVAL;
    if (kind == 4) { // copy at RCCL's transport-kernel footprint (k_fatcopy)
        hipLaunchKernelGGL(k_fatcopy, dim3(blocks), dim3(256), 0, st, out, a, n / 2);
        return launch_status();
    }
    using K = void (*)(double*, const double*, const double*, int64_t, double*);
    if (blocks <= 0) { // the flat grid (k_bwflat): unroll 1, 2 or 4 dwordx4 per thread
        static const K flat[4][3][2] = {
#define GS_BWF(KD) {{k_bwflat<KD, 1, false>, k_bwflat<KD, 1, true>}, {k_bwflat<KD, 2, false>, k_bwflat<KD, 2, true>}, \
                    {k_bwflat<KD, 4, false>, k_bwflat<KD, 4, true>}}
            GS_BWF(0), GS_BWF(1), GS_BWF(2), GS_BWF(3)
#undef GS_BWF
        };
        const int u = unroll >= 4 ? 2 : (unroll >= 2 ? 1 : 0);
        const int64_t per = 256LL << u, nb = (n / 2 + per - 1) / per;
        if (nb <= 0 || nb > 0x7fffffff) return nb <= 0 ? 0 : GS_EINVAL;
        hipLaunchKernelGGL(flat[kind][u][nt != 0], dim3((unsigned)nb), dim3(256), 0, st, out, a, b, n / 2, sink);
        return launch_status();
    }
    static const K tab[4][2][2] = {
        {{k_bw<0, 1, false>, k_bw<0, 1, true>}, {k_bw<0, 4, false>, k_bw<0, 4, true>}},
        {{k_bw<1, 1, false>, k_bw<1, 1, true>}, {k_bw<1, 4, false>, k_bw<1, 4, true>}},
        {{k_bw<2, 1, false>, k_bw<2, 1, true>}, {k_bw<2, 4, false>, k_bw<2, 4, true>}},
        {{k_bw<3, 1, false>, k_bw<3, 1, true>}, {k_bw<3, 4, false>, k_bw<3, 4, true>}},
    };
    hipLaunchKernelGGL(tab[kind][unroll > 1][nt != 0], dim3(blocks), dim3(256), 0, st, out, a, b, n / 2, sink);
    return launch_status();
}

int gs_debug_march(int pfd, int bar, int nts, int ntf, int zc, const gs_level* L, const double* v, const double* f,
                   double* out, hipStream_t st)
{
    if (!L || bad_level(L) || !v || !f || !out || zc < 1 || (pfd != 1 && pfd != 2) || L->nx > 512 || L->ny % 4)
        return GS_EINVAL;
    if (ntf >= 6) { // (ntf 6 / 7: RY = 1 / 4 rows per wave, 2 / 8-row tiles; pfd 2, barrier, nt stores)
        const int ry = ntf == 6 ? 1 : 4;
        if (L->ny % (2 * ry)) return GS_EINVAL;
        const dim3 g((unsigned)(L->ny / (2 * ry)), (unsigned)((L->nz + zc - 1) / zc)), b(WAVE, 4, 2);
        if (ry == 1) hipLaunchKernelGGL((k_march<2, true, true, false, false, 0, 1>), g, b, 0, st, v, f, out,
                                        (int)L->nx, (int)L->ny, (int)L->nz, L->ldy, L->ldz, zc, nullptr);
        else hipLaunchKernelGGL((k_march<1, true, true, false, false, 0, 4>), g, b, 0, st, v, f, out, (int)L->nx,
                                (int)L->ny, (int)L->nz, L->ldy, L->ldz, zc, nullptr);
        return launch_status();
    }
    if (ntf >= 3) { // (ntf 3 / 4 / 5: bounded drift of 2 / 4 / 8 plane steps, pfd 2, barrier, nt stores; the counter
                    // lives in out's plane -1, zeroed here)
        const dim3 g((unsigned)(L->ny / 4), (unsigned)((L->nz + zc - 1) / zc)), b(WAVE, 4, 2);
        if ((int64_t)g.x * g.y > 256) return GS_EINVAL; // (every block must be resident: one per CU)
        unsigned* cnt = reinterpret_cast<unsigned*>(out - L->ldz); // (plane -1 of the padded layout)
        if (hipMemsetAsync(cnt, 0, 16, st) != hipSuccess) return GS_EINVAL;
#define GS_MS(D) hipLaunchKernelGGL((k_march<2, true, true, false, false, D>), g, b, 0, st, v, f, out, (int)L->nx, \
                                    (int)L->ny, (int)L->nz, L->ldy, L->ldz, zc, cnt)
        if (ntf == 3) GS_MS(2); else if (ntf == 4) GS_MS(4); else GS_MS(8);
#undef GS_MS
        return launch_status();
    }
    if (ntf >= 2) { // (ntf 2: LEAN loads, pfd 2, nt stores)
        const dim3 g((unsigned)(L->ny / 4), (unsigned)((L->nz + zc - 1) / zc)), b(WAVE, 4, 2);
        if (bar) hipLaunchKernelGGL((k_march<2, true, true, false, true>), g, b, 0, st, v, f, out, (int)L->nx,
                                    (int)L->ny, (int)L->nz, L->ldy, L->ldz, zc, nullptr);
        else hipLaunchKernelGGL((k_march<2, false, true, false, true>), g, b, 0, st, v, f, out, (int)L->nx,
                                (int)L->ny, (int)L->nz, L->ldy, L->ldz, zc, nullptr);
        return launch_status();
    }
    using K = void (*)(const double*, const double*, double*, int, int, int, int64_t, int64_t, int, unsigned*);
    static const K tab[2][2][2][2] = {
#define GS_MF(P, B) {{k_march<P, B, false, false>, k_march<P, B, false, true>}, \
                     {k_march<P, B, true, false>, k_march<P, B, true, true>}}
        {GS_MF(1, false), GS_MF(1, true)}, {GS_MF(2, false), GS_MF(2, true)}
#undef GS_MF
    };
    const dim3 g((unsigned)(L->ny / 4), (unsigned)((L->nz + zc - 1) / zc)), b(WAVE, 4, 2);
    hipLaunchKernelGGL(tab[pfd - 1][bar != 0][nts != 0][ntf != 0], g, b, 0, st, v, f, out, (int)L->nx, (int)L->ny,
                       (int)L->nz, L->ldy, L->ldz, zc, nullptr);
    return launch_status();
}

int gs_debug_phase_probe(int work, int threads, int phases, double* g, double* sink, hipStream_t st)
{
    if ((threads != 512 && threads != 1024) || phases < 0 || work < 0 || work > 2 || !g || !sink) return GS_EINVAL;
    if (work == 0) hipLaunchKernelGGL(k_phase_probe<0>, dim3(1), dim3(threads), 0, st, g, phases, sink);
    else if (work == 1) hipLaunchKernelGGL(k_phase_probe<1>, dim3(1), dim3(threads), 0, st, g, phases, sink);
    else hipLaunchKernelGGL(k_phase_probe<2>, dim3(1), dim3(threads), 0, st, g, phases, sink);
    return launch_status();
}

int gs_debug_div_check(const double* a, int64_t n, double hh, double* fast, double* ref, hipStream_t st)
{
    if (!a || !fast || !ref || n < 0) return GS_EINVAL;
    if (n == 0) return 0;
    Coef k{};
    k.hh = hh;
    k.fastdiv = hh >= 0x1p-120 && hh <= 1.0;
    hipLaunchKernelGGL(k_div_check, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, n, k, fast, ref);
    return launch_status();
}

int gs_debug_nb_quot(const double* r, const double* den, int64_t n, double* q, hipStream_t st)
{
    if (!r || !den || !q || n < 0) return GS_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_nb_quot, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, r, den, n, q);
    return launch_status();
}

int gs_debug_stream_triad(double* out, const double* a, const double* b, int64_t n, hipStream_t st)
{
    if (!out || !a || !b || n < 0 || (n & 1)) return GS_EINVAL;
    hipLaunchKernelGGL(k_triad, dim3(4096), dim3(256), 0, st, out, a, b, n / 2);
    return launch_status();
}

} // extern "C"
