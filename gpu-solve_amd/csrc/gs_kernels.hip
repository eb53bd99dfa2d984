// gs_kernels.hip — the product library libgpusolve_hip.so: the extern "C" launchers declared in
// include/gpusolve_hip.h over the gfx950 kernels of gs_device.hpp. Diagnostics (tuning variants,
// bandwidth probes, the rejected k_prr) live in gs_diag.hip -> libgpusolve_diag.so.
#include "gs_device.hpp"

// =============================================================================================
extern "C" {

int gs_field_layout(int64_t nx, int64_t ny, int64_t nz, int64_t* ldy, int64_t* ldz, int64_t* alloc_elems,
                    int64_t* origin_offset)
{
    if (nx < 0 || ny < 0 || nz < 0 || !ldy || !ldz || !alloc_elems || !origin_offset) return GS_EINVAL;
    // x=1 of every row 128-B aligned: pitch a multiple of 16 doubles, origin at 15 (mod 16).
    const int64_t py = ((nx + 2 + 15) / 16) * 16;
    *ldy = py;
    *ldz = py * (ny + 2);
    // one extra plane below plane 0 and above plane nz+1 (Z-slab ghost depth 2 for the fused
    // two-sweep kernel), plus slack for the clamped pair loads at the last row
    *origin_offset = 15 + *ldz;
    *alloc_elems = *ldz * (nz + 4) + 32;
    return 0;
}

int gs_rhs_init(const gs_level* L, double* f, int mode, double h0, double gamma, hipStream_t st)
{
    if (bad_level(L) || !f) return GS_EINVAL;
    const dim3 g((unsigned)((L->nx + 2 + 63) / 64), (unsigned)((L->ny + 2 + 3) / 4), (unsigned)(L->nz + 2)), b(64, 4);
    hipLaunchKernelGGL(k_rhs, g, b, 0, st, f, mode, h0, gamma, (int)L->nx, (int)L->ny, (int)L->nz, L->z0, L->ldy,
                       L->ldz);
    return launch_status();
}

int gs_jacobi_sweep(const gs_stencil* S, const gs_level* L, int mode, double omega, double gamma,
                    const double* v_in, double* v_out, const double* f, const double* w, hipStream_t st)
{
    return gs_jacobi_sweep_norm(S, L, mode, omega, gamma, v_in, v_out, f, w, nullptr, st);
}

int gs_jacobi_sweep_norm(const gs_stencil* S, const gs_level* L, int mode, double omega, double gamma,
                         const double* v_in, double* v_out, const double* f, const double* w, double* partials,
                         hipStream_t st)
{
    mode = base_mode(mode);
    if (!v_out || !f || v_in == v_out || (newtonish(mode) && !w)) return GS_EINVAL;
    if (partials && L && (L->nx == 0 || L->ny == 0 || L->nz == 0))
        return (int)hipMemsetAsync(partials, 0, sizeof(double), st);
    return launch_pass<0, false>(S, L, mode, omega, gamma, v_in, f, w, v_out, partials, st);
}

int gs_jacobi_sweep2_supported_mode(const gs_stencil* S, const gs_level* L, int mode)
{
    int zc;
    dim3 g, b;
    mode = base_mode(mode);
    if (mode < GS_LINEAR || mode > GS_NEWTON_B) return 0;
    return (!bad_level(L) && valid_stencil(S)) ? tb2_plan(S, L, &zc, &g, &b, nullptr, mode) : 0;
}

int gs_jacobi_sweep2_supported(const gs_stencil* S, const gs_level* L)
{
    int r = 2;
    for (int m = GS_LINEAR; m <= GS_NEWTON; m++) {
        const int q = gs_jacobi_sweep2_supported_mode(S, L, m);
        r = q < r ? q : r;
    }
    return r;
}

int gs_jacobi_sweep2(const gs_stencil* S, const gs_level* L, int mode, double omega, double gamma,
                     const double* v_in, double* v_out, const double* f, const double* w, int zlo, int zhi,
                     hipStream_t st)
{
    return gs_jacobi_sweep2_norm(S, L, mode, omega, gamma, v_in, v_out, f, w, zlo, zhi, nullptr, st);
}

const char* gs_jacobi_sweep2_kernel(const gs_stencil* S, const gs_level* L, int mode)
{
    int zc;
    dim3 g, b;
    bool y2 = false, xh = false;
    mode = base_mode(mode);
    if (bad_level(L) || !valid_stencil(S) || !tb2_plan(S, L, &zc, &g, &b, &y2, mode, &xh)) return "";
    if (y2) return "k_tb2y: 4x2 waves, 2 rows per wave, LDS halo-row exchange, per-wave-row code";
    if (xh) return "k_tb2y XH: 512-point column blocks of 4x2 waves, edge columns computed lane-parallel";
    return "k_tb2: <= 8 x-waves, 2 rows per wave";
}

int64_t gs_jacobi_sweep2_num_partials(const gs_stencil* S, const gs_level* L, int mode)
{
    int zc;
    dim3 g, b;
    mode = base_mode(mode);
    if (bad_level(L) || !valid_stencil(S) || !tb2_plan(S, L, &zc, &g, &b, nullptr, mode)) return 0;
    return (int64_t)g.x * g.y;
}

int gs_jacobi_sweep2_norm(const gs_stencil* S, const gs_level* L, int mode, double omega, double gamma,
                          const double* v_in, double* v_out, const double* f, const double* w, int zlo, int zhi,
                          double* partials, hipStream_t st)
{
    int zc;
    dim3 g, b;
    bool y2 = false, xh = false;
    // GS_NEWTON_G: the GS_NEWTON_B kernels take gamma for the factor instead of loading it (Coef::bconst)
    const int bconst = mode == GS_NEWTON_G;
    mode = base_mode(mode);
    if (!S || bad_level(L) || !valid_stencil(S) || !v_out || !f || v_in == v_out || (!v_in && mode == GS_NONLINEAR) ||
        (newtonish(mode) && !w) || mode < GS_LINEAR || mode > GS_NEWTON_B ||
        !tb2_plan(S, L, &zc, &g, &b, &y2, mode, &xh))
        return GS_EINVAL;
    const Coef k = make_coef(S, L, omega, gamma, bconst);
    const int nx = (int)L->nx, ny = (int)L->ny, nz = (int)L->nz;
#define GS_TB(M, Z) hipLaunchKernelGGL((k_tb2<M, TB_RY_B, TB_WX_B, true, false, Z>), g, b, 0, st, k, v_in, f, w, v_out, partials, nx, ny, nz, L->ldy, L->ldz, zc, zlo ? 1 : 0, zhi ? 1 : 0, nullptr, nullptr, 0, 0, 0, 0, 0, nullptr)
    // LINEAR zero-iterate pairs (the first sweep of a coarse level, v = 0: the lightest variant, three
    // blocks per CU) below 2^26 points: chunks fitted to whole rounds of resident blocks (256^3: 61 vs
    // 71 us; the same rule measured no better for the other pairs, worse for k_rr2 and for NEWTON's
    // zero-iterate pair at two blocks per CU: 133 vs 120 us, r02 tools/fit_session.sh)
    const bool refit = !v_in && !partials && (int64_t)L->nx * L->ny * L->nz < ((int64_t)1 << 26);
    // GS_SPEC_CACHED=1: pairs with norm partials (the V-cycle's speculative pre-smoothing pair, which k_rr2 reads
    // next, last planes first) store through the caches instead of non-temporally (A/B)
    const bool cached = partials && kKnobs.specCached;
#define GS_TBY2(M, Z, U, P) do { \
        if (refit && M == GS_LINEAR) refit_chunks(&k_tb2y<M, newtonish(M) ? TBY_RY_NEWTON : TBY_RY, TBY_WX, true, false, Z, true, 0, P, false, U>, (int)(b.x * b.y * b.z), nz, 4, 64, true, 2.0, &zc, &g); \
        if (cached) hipLaunchKernelGGL((k_tb2y<M, newtonish(M) ? TBY_RY_NEWTON : TBY_RY, TBY_WX, false, false, Z, true, 0, P, false, U>), g, b, 0, st, k, v_in, f, w, v_out, partials, nx, ny, nz, L->ldy, L->ldz, zc, zlo ? 1 : 0, zhi ? 1 : 0, nullptr, nullptr, 0, 0, 0, 0, 0, nullptr); \
        else hipLaunchKernelGGL((k_tb2y<M, newtonish(M) ? TBY_RY_NEWTON : TBY_RY, TBY_WX, true, false, Z, true, 0, P, false, U>), g, b, 0, st, k, v_in, f, w, v_out, partials, nx, ny, nz, L->ldy, L->ldz, zc, zlo ? 1 : 0, zhi ? 1 : 0, nullptr, nullptr, 0, 0, 0, 0, 0, nullptr); } while (0)
#define GS_TBY1(M, Z, U) GS_TBY2(M, Z, U, tby_pfd(M))
#define GS_TBY(M, Z) do { if (k.unit) GS_TBY1(M, Z, true); else GS_TBY1(M, Z, false); } while (0)
#define GS_TBX1(M, Z, P, U) hipLaunchKernelGGL((k_tb2y<M, TBY_RY, TBY_WX, true, false, Z, true, 0, P, true, U>), g, b, 0, st, k, v_in, f, w, v_out, partials, nx, ny, nz, L->ldy, L->ldz, zc, zlo ? 1 : 0, zhi ? 1 : 0, nullptr, nullptr, 0, 0, 0, 0, 0, nullptr)
#define GS_TBX(M, Z, P) do { if (k.unit) GS_TBX1(M, Z, P, true); else GS_TBX1(M, Z, P, false); } while (0)
    const bool zv = !v_in;
    // FX (r06): LINEAR plain pairs over rows of whole 128-point waves (512-point column blocks) take the instance
    // without per-lane range selects (k_tb2y FX; GS_PAIR_FX=0: the general instance, A/B)
    if (mode == GS_LINEAR && !zv && k.unit && kKnobs.pairFx &&
        ((xh && tbx_pfd2() && nx % (2 * WAVE * TBY_WX) == 0) || (y2 && nx % (2 * WAVE) == 0))) {
        if (xh)
            hipLaunchKernelGGL((k_tb2y<GS_LINEAR, TBY_RY, TBY_WX, true, false, false, true, 0, 2, true, true, false, 0, true>),
                               g, b, 0, st, k, v_in, f, w, v_out, partials, nx, ny, nz, L->ldy, L->ldz, zc, zlo ? 1 : 0,
                               zhi ? 1 : 0, nullptr, nullptr, 0, 0, 0, 0, 0, nullptr);
        else if (cached)
            hipLaunchKernelGGL((k_tb2y<GS_LINEAR, TBY_RY, TBY_WX, false, false, false, true, 0, 2, false, true, false, 0, true>),
                               g, b, 0, st, k, v_in, f, w, v_out, partials, nx, ny, nz, L->ldy, L->ldz, zc, zlo ? 1 : 0,
                               zhi ? 1 : 0, nullptr, nullptr, 0, 0, 0, 0, 0, nullptr);
        else
            hipLaunchKernelGGL((k_tb2y<GS_LINEAR, TBY_RY, TBY_WX, true, false, false, true, 0, 2, false, true, false, 0, true>),
                               g, b, 0, st, k, v_in, f, w, v_out, partials, nx, ny, nz, L->ldy, L->ldz, zc, zlo ? 1 : 0,
                               zhi ? 1 : 0, nullptr, nullptr, 0, 0, 0, 0, 0, nullptr);
    } else if (mode == GS_NEWTON_B && !zv && y2 && !cached && k.unit && kKnobs.pairFx && nx % (2 * WAVE) == 0) {
        hipLaunchKernelGGL((k_tb2y<GS_NEWTON_B, TBY_RY_NEWTON, TBY_WX, true, false, false, true, 0, 1, false, true, false, 0, true>),
                           g, b, 0, st, k, v_in, f, w, v_out, partials, nx, ny, nz, L->ldy, L->ldz, zc, zlo ? 1 : 0,
                           zhi ? 1 : 0, nullptr, nullptr, 0, 0, 0, 0, 0, nullptr);
    } else if (xh) {
        if (mode == GS_LINEAR) {
            if (zv) GS_TBX(GS_LINEAR, true, 1);
            else if (tbx_pfd2()) GS_TBX(GS_LINEAR, false, 2);
            else GS_TBX(GS_LINEAR, false, 1);
        } else if (mode == GS_NONLINEAR) GS_TBX(GS_NONLINEAR, false, 1);
        else if (mode == GS_NEWTON_B && zv) GS_TBX(GS_NEWTON_B, true, 1);
        else if (mode == GS_NEWTON_B) GS_TBX(GS_NEWTON_B, false, 1);
        else if (zv) GS_TBX(GS_NEWTON, true, 1);
        else GS_TBX(GS_NEWTON, false, 1);
    } else if (y2) {
        if (mode == GS_LINEAR) {
            if (zv) GS_TBY(GS_LINEAR, true);
            else GS_TBY(GS_LINEAR, false);
        } else if (mode == GS_NONLINEAR) GS_TBY(GS_NONLINEAR, false);
        else if (mode == GS_NEWTON_B && zv) GS_TBY(GS_NEWTON_B, true);
        else if (mode == GS_NEWTON_B) GS_TBY(GS_NEWTON_B, false);
        else if (zv) GS_TBY(GS_NEWTON, true);
        else GS_TBY(GS_NEWTON, false);
    } else {
        if (mode == GS_LINEAR) {
            if (zv) GS_TB(GS_LINEAR, true);
            else GS_TB(GS_LINEAR, false);
        } else if (mode == GS_NONLINEAR) GS_TB(GS_NONLINEAR, false);
        else if (mode == GS_NEWTON_B && zv) GS_TB(GS_NEWTON_B, true);
        else if (mode == GS_NEWTON_B) GS_TB(GS_NEWTON_B, false);
        else if (zv) GS_TB(GS_NEWTON, true);
        else GS_TB(GS_NEWTON, false);
    }
#undef GS_TBX
#undef GS_TBX1
#undef GS_TBY
#undef GS_TBY1
#undef GS_TBY2
#undef GS_TB
    return launch_status();
}

int gs_jacobi_sweep2_prolong_supported(const gs_stencil* S, const gs_level* L, int mode)
{
    int zc;
    dim3 g, b;
    bool y2 = false, xh = false;
    mode = base_mode(mode);
    // LINEAR and NEWTON (NONLINEAR carries restV too). Rows of more than 512 points (column blocks, XH,
    // NEWTON too since r04) with the workspace of gs_jacobi_sweep2_prolong_ws_elems (the corrected edge
    // columns). The fine planes' parities must be the global ones (even z0): they select each plane's
    // combination
    return !bad_level(L) && valid_stencil(S) && (mode == GS_LINEAR || newtonish(mode)) && L->z0 % 2 == 0 &&
           tb2_plan(S, L, &zc, &g, &b, &y2, mode, &xh, true) && (y2 || xh);
}

int64_t gs_jacobi_sweep2_prolong_ws_elems(const gs_stencil* S, const gs_level* L, int mode)
{
    int zc;
    dim3 g, b;
    bool y2 = false, xh = false;
    mode = base_mode(mode);
    if (!gs_jacobi_sweep2_prolong_supported(S, L, mode) || !tb2_plan(S, L, &zc, &g, &b, &y2, mode, &xh, true) || !xh)
        return 0;
    const int64_t bw = 2 * WAVE * TBY_WX, nb = (L->nx + bw - 1) / bw - 1; // interior block boundaries
    return nb * (L->nz + 4) * 4 * (L->ny + 2);
}

int gs_jacobi_sweep2_prolong(const gs_stencil* S, const gs_level* L, int mode, double omega, double gamma,
                             const double* v_in, const double* coarse_v, const double* coarse_sub, const gs_level* cl,
                             double* v_out, const double* f, const double* w, int zlo, int zhi, hipStream_t st)
{
    return gs_jacobi_sweep2_prolong_ws(S, L, mode, omega, gamma, v_in, coarse_v, coarse_sub, cl, v_out, f, w, zlo, zhi,
                                       nullptr, 0, st);
}

int gs_jacobi_sweep2_prolong_ws(const gs_stencil* S, const gs_level* L, int mode, double omega, double gamma,
                                const double* v_in, const double* coarse_v, const double* coarse_sub,
                                const gs_level* cl, double* v_out, const double* f, const double* w, int zlo, int zhi,
                                double* ws, int64_t ws_elems, hipStream_t st)
{
    int zc;
    dim3 g, b;
    bool y2 = false, xh = false;
    const int bconst = mode == GS_NEWTON_G; // (Coef::bconst, as gs_jacobi_sweep2_norm)
    mode = base_mode(mode);
    // coarse plane of fine local plane z: (z >> 1) + czoff, z0 even (a slab, or a plane range of one)
    const int64_t czoff = cl ? L->z0 / 2 - cl->z0 : 0;
    if (!gs_jacobi_sweep2_prolong_supported(S, L, mode) || bad_level(cl) || czoff < 0 || !v_in || !coarse_v ||
        !v_out || !f || v_in == v_out || (mode == GS_NONLINEAR) != (coarse_sub != nullptr) || (newtonish(mode) && !w) ||
        (L->nx + 1) / 2 > cl->nx + 1 || (L->ny + 1) / 2 > cl->ny + 1 || (L->nz + 1) / 2 + czoff > cl->nz + 1 ||
        !tb2_plan(S, L, &zc, &g, &b, &y2, mode, &xh, true))
        return GS_EINVAL;
    const int64_t need = gs_jacobi_sweep2_prolong_ws_elems(S, L, mode);
    if (need > 0 && (!ws || ws_elems < need)) return GS_EINVAL;
    // the kernel indexes the coarse field from the plane under fine local plane 0
    coarse_v += czoff * cl->ldz;
    if (coarse_sub) coarse_sub += czoff * cl->ldz;
    const Coef k = make_coef(S, L, omega, gamma, bconst);
    if (xh && need > 0) {
        const int bw = 2 * WAVE * TBY_WX, nb = (int)((L->nx + bw - 1) / bw - 1);
        hipLaunchKernelGGL(k_pro_strip<false>, dim3((unsigned)((L->ny + 2 + 63) / 64), (unsigned)(L->nz + 4), (unsigned)nb),
                           dim3(256), 0, st, v_in, coarse_v, nullptr, ws, (int)L->nx, (int)L->ny, (int)L->nz, L->ldy,
                           L->ldz, cl->ldy, cl->ldz, bw, zlo ? 1 : 0, zhi ? 1 : 0);
    }
#define GS_TBPF(M, P, U, X, WM, FXV) hipLaunchKernelGGL((k_tb2y<M, newtonish(M) ? TBY_RY_NEWTON : TBY_RY, WM, true, false, false, true, P, 1, X, U, false, 0, FXV>), g, b, 0, st, k, v_in, f, w, v_out, nullptr, (int)L->nx, (int)L->ny, (int)L->nz, L->ldy, L->ldz, zc, zlo ? 1 : 0, zhi ? 1 : 0, coarse_v, coarse_sub, (int)cl->nx, (int)cl->ny, (int)(cl->nz - czoff), cl->ldy, cl->ldz, ws)
    // FX (r06, as the plain pairs): unit-stencil LINEAR / GS_NEWTON_B prolongation pairs of four x-waves over rows of
    // whole 128-point waves (512-point column blocks) take the instance without per-lane range selects
    const bool fx = k.unit && kKnobs.pairFx && b.y == TBY_WX && (xh ? L->nx % (2 * WAVE * TBY_WX) == 0 : L->nx % (2 * WAVE) == 0);
#define GS_TBP1(M, P, U, X, WM) do { \
        if constexpr (U && WM == TBY_WX && (M == GS_LINEAR || M == GS_NEWTON_B)) { \
            if (fx) GS_TBPF(M, P, U, X, WM, true); \
            else GS_TBPF(M, P, U, X, WM, false); \
        } else { \
            GS_TBPF(M, P, U, X, WM, false); \
        } } while (0)
#define GS_TBP(M, P, X, WM) do { if (k.unit) GS_TBP1(M, P, true, X, WM); else GS_TBP1(M, P, false, X, WM); } while (0)
    // NEWTON's variant keeps ~37 KB of state per x-wave in LDS (its RECOMP rows): rows of <= 256 points
    // (two x-waves) take the instance sized for two, so that two blocks share a CU (8 waves, the VGPR
    // limit) instead of one block of 4 waves holding the whole LDS of a four-x-wave instance
    // (NEWTON column blocks: the RECOMP LDS state and the edge columns together, 144 B per lane spilled)
    if (mode == GS_NEWTON_B && xh) GS_TBP(GS_NEWTON_B, 1, true, TBY_WX);
    else if (mode == GS_NEWTON_B && b.y <= 2) GS_TBP(GS_NEWTON_B, 1, false, 2);
    else if (mode == GS_NEWTON_B) GS_TBP(GS_NEWTON_B, 1, false, TBY_WX);
    else if (mode == GS_NEWTON && xh) GS_TBP(GS_NEWTON, 1, true, TBY_WX);
    else if (mode == GS_NEWTON && b.y <= 2) GS_TBP(GS_NEWTON, 1, false, 2);
    else if (mode == GS_NEWTON) GS_TBP(GS_NEWTON, 1, false, TBY_WX);
    else if (xh) GS_TBP(GS_LINEAR, 1, true, TBY_WX);
    else GS_TBP(GS_LINEAR, 1, false, TBY_WX);
#undef GS_TBP
#undef GS_TBPF
#undef GS_TBP1
    return launch_status();
}

// the small-level tiled kernels (gs_device.hpp k_tile_*): LINEAR / NEWTON, canonical stencil order, whole levels
int gs_tiled_supported(const gs_stencil* S, const gs_level* L, int mode)
{
    mode = base_mode(mode);
    return S && valid_stencil(S) && canonical_order(S) && (mode == GS_LINEAR || newtonish(mode)) && !bad_level(L) &&
           L->z0 == 0 && L->nx >= 1 && L->ny >= 1 && L->nz >= 1;
}

int gs_smooth2_restrict_tiled(const gs_stencil* S, const gs_level* fl, int mode, double omega, double gamma,
                              const double* v_in, double* v_out, const double* f, const double* w, double* coarse_f,
                              const gs_level* cl, hipStream_t st)
{
    mode = base_mode(mode); // (the tiled kernels read the factor field, which holds gamma under GS_NEWTON_G)
    if (!gs_tiled_supported(S, fl, mode) || bad_level(cl) || cl->z0 != 0 || !v_out || !f || !coarse_f ||
        v_in == v_out || (newtonish(mode) && !w) || cl->nx != fl->nx / 2 || cl->ny != fl->ny / 2 ||
        cl->nz != fl->nz / 2)
        return GS_EINVAL;
    const Coef k = make_coef(S, fl, omega, gamma);
    const dim3 g((unsigned)((fl->nx + TS - 1) / TS), (unsigned)((fl->ny + TS - 1) / TS), (unsigned)((fl->nz + TS - 1) / TS));
#define GS_TPR(M, Z, U) hipLaunchKernelGGL((k_tile_pre_rr<M, Z, U>), g, dim3(TS_T), 0, st, k, v_in, f, w, v_out, coarse_f, (int)fl->nx, (int)fl->ny, (int)fl->nz, fl->ldy, fl->ldz, (int)cl->nx, (int)cl->ny, (int)cl->nz, cl->ldy, cl->ldz)
#define GS_TPRM(M) do { \
        if (!v_in) { if (k.unit) GS_TPR(M, true, true); else GS_TPR(M, true, false); } \
        else { if (k.unit) GS_TPR(M, false, true); else GS_TPR(M, false, false); } } while (0)
    if (mode == GS_NEWTON_B) GS_TPRM(GS_NEWTON_B);
    else if (mode == GS_NEWTON) GS_TPRM(GS_NEWTON);
    else GS_TPRM(GS_LINEAR);
#undef GS_TPRM
#undef GS_TPR
    return launch_status();
}

int gs_prolong_smooth2_tiled(const gs_stencil* S, const gs_level* fl, int mode, double omega, double gamma,
                             const double* v_in, const double* coarse_v, const gs_level* cl, double* v_out,
                             const double* f, const double* w, hipStream_t st)
{
    mode = base_mode(mode);
    if (!gs_tiled_supported(S, fl, mode) || bad_level(cl) || cl->z0 != 0 || !v_in || !coarse_v || !v_out || !f ||
        v_in == v_out || (newtonish(mode) && !w) || (fl->nx + 1) / 2 > cl->nx + 1 || (fl->ny + 1) / 2 > cl->ny + 1 ||
        (fl->nz + 1) / 2 > cl->nz + 1)
        return GS_EINVAL;
    const Coef k = make_coef(S, fl, omega, gamma);
    const dim3 g((unsigned)((fl->nx + TS - 1) / TS), (unsigned)((fl->ny + TS - 1) / TS), (unsigned)((fl->nz + TS - 1) / TS));
#define GS_TP2(M, U) hipLaunchKernelGGL((k_tile_pro2<M, U>), g, dim3(TS_T), 0, st, k, v_in, coarse_v, f, w, v_out, (int)fl->nx, (int)fl->ny, (int)fl->nz, fl->ldy, fl->ldz, cl->ldy, cl->ldz)
    if (mode == GS_NEWTON_B) {
        if (k.unit) GS_TP2(GS_NEWTON_B, true);
        else GS_TP2(GS_NEWTON_B, false);
    } else if (mode == GS_NEWTON) {
        if (k.unit) GS_TP2(GS_NEWTON, true);
        else GS_TP2(GS_NEWTON, false);
    } else {
        if (k.unit) GS_TP2(GS_LINEAR, true);
        else GS_TP2(GS_LINEAR, false);
    }
#undef GS_TP2
    return launch_status();
}

int64_t gs_residual_num_partials(const gs_stencil* S, const gs_level* L)
{
    if (!S || !L) return 0;
    if (L->nx == 0 || L->ny == 0 || L->nz == 0) return 1;
    const dim3 g = pass_plan(S, L).grid;
    return (int64_t)g.x * g.y * g.z;
}

int gs_residual(const gs_stencil* S, const gs_level* L, int mode, double gamma, const double* v, const double* f,
                const double* w, double* r, double* partials, hipStream_t st)
{
    mode = base_mode(mode);
    if (!f || (newtonish(mode) && !w)) return GS_EINVAL;
    if (partials && (L && (L->nx == 0 || L->ny == 0 || L->nz == 0)))
        return (int)hipMemsetAsync(partials, 0, sizeof(double), st);
    return launch_pass<1, false>(S, L, mode, 0.0, gamma, v, f, w, r, partials, st);
}

int gs_sumsq_finish(const double* partials, int64_t n, double* out, int accumulate, hipStream_t st)
{
    if (!partials || !out || n < 0) return GS_EINVAL;
    hipLaunchKernelGGL(k_sumsq_finish, dim3(1), dim3(FIN_T), 0, st, partials, n, out, accumulate);
    return launch_status();
}

int gs_restrict2(const double* fine, const gs_level* fl, double* ca, double* cb, const gs_level* cl, hipStream_t st)
{
    if (!fine || !ca || bad_level(fl) || bad_level(cl)) return GS_EINVAL;
    if (cl->nx == 0 || cl->ny == 0 || cl->nz == 0) return 0;
    const int64_t zoff = 2 * cl->z0 - fl->z0; // fine local centre plane = 2 z + zoff
    if (2 * cl->nx + 1 > fl->nx + 1 || 2 * cl->ny + 1 > fl->ny + 1 || 2 + zoff - 1 < 0 ||
        2 * cl->nz + zoff + 1 > fl->nz + 1)
        return GS_EINVAL;
    const dim3 g((unsigned)((cl->nx + 63) / 64), (unsigned)((cl->ny + 3) / 4), (unsigned)cl->nz), b(64, 4);
    hipLaunchKernelGGL(k_restrict, g, b, 0, st, fine, ca, cb, (int)cl->nx, (int)cl->ny, (int)cl->nz, fl->ldy, fl->ldz,
                       cl->ldy, cl->ldz, (int)zoff);
    return launch_status();
}

int gs_residual_restrict(const gs_stencil* S, const gs_level* fl, int mode, double gamma, const double* v,
                         const double* f, const double* w, double* ca, double* cb, const gs_level* cl, hipStream_t st)
{
    return gs_residual_restrict_slab(S, fl, mode, gamma, v, f, w, ca, cb, cl, 0, st);
}

int gs_residual_restrict_slab_supported(const gs_stencil* S, const gs_level* fl)
{
    const bool ldsOnly = kKnobs.rrLds;
    return S && fl && !bad_level(fl) && valid_stencil(S) && canonical_order(S) && !ldsOnly &&
           ((fl->nx + 1) / 2 + WAVE - 1) / WAVE <= RR2_WXMAX;
}

int gs_residual_restrict_slab(const gs_stencil* S, const gs_level* fl, int mode, double gamma, const double* v,
                              const double* f, const double* w, double* ca, double* cb, const gs_level* cl, int zhi,
                              hipStream_t st)
{
    const int bconst = mode == GS_NEWTON_G; // (Coef::bconst: k_rr2 takes gamma for the factor)
    mode = base_mode(mode);
    if (!S || !valid_stencil(S) || !v || !f || !ca || (newtonish(mode) && !w) || mode < GS_LINEAR ||
        mode > GS_NEWTON_B || bad_level(fl) || bad_level(cl))
        return GS_EINVAL;
    if (cl->nx == 0 || cl->ny == 0 || cl->nz == 0) return 0;
    const int64_t zoff = 2 * cl->z0 - fl->z0; // fine local centre plane = 2 z + zoff
    // the residual is evaluated on fine local planes 2z+zoff-1 .. 2z+zoff+1 of the interior only
    // (planes 0 and nz+1 hold r = 0): they must exist, as must the coarse points' fine columns
    if (2 * cl->nx + 1 > fl->nx + 1 || 2 * cl->ny + 1 > fl->ny + 1 || 2 + zoff - 1 < 0 ||
        2 * cl->nz + zoff + 1 > fl->nz + 1)
        return GS_EINVAL;
    const Coef k = make_coef(S, fl, 0.0, gamma, bconst);
    const int64_t wxs = ((fl->nx + 1) / 2 + WAVE - 1) / WAVE; // x-waves covering coarse columns 1..(fnx+1)/2
    const bool ldsOnly = kKnobs.rrLds; // A/B switch for tools/ measurements
    const bool rr2 = !ldsOnly && canonical_order(S) && zoff == 0 && wxs <= RR2_WXMAX;
    if (zhi && !rr2) return GS_EINVAL; // the slab form exists for the register kernel only
    // the LDS-DMA ring form (k_rr2d): rows of up to 4 x-waves (fine rows <= 512 points) whose lanes never clamp a
    // column (every lane's dwordx4 lies inside the padded row). GS_RR_DMA: 0 never (default), 1 the factor-loading
    // GS_NEWTON_B launches only, 2 every eligible launch (A/B). Measured slower where it matters (r06):
    // alone, 512^3 LINEAR 0.533-0.540 vs 0.459 ms, NEWTON_B 0.710-0.712 vs 0.726 ms, GS_NEWTON_G 0.576 vs 0.494 ms;
    // in the Newton cycle (GS_RR_DMA=1) 29.26 / 29.40 vs 28.58 / 28.55 ms per iteration. One block per CU (the ring
    // takes 132-144 KB) and LDS-DMA's landing rate, ~25-32 GB/s per CU measured here (MI355X_MICROARCH.md
    // 'ldsdma-fill': ~25 GB/s per CU), cap it below what two register-loading blocks per CU reach
    const bool dmaMode = kKnobs.rrDma >= 2 || (kKnobs.rrDma == 1 && mode == GS_NEWTON_B && !bconst);
    const bool dma = rr2 && dmaMode && wxs <= RR2D_WXMAX && 2 * WAVE * wxs - 1 <= fl->nx + 1;
    if (dma) {
        const bool big = fl->nx * fl->ny * fl->nz >= ((int64_t)1 << RR2_NR2_LOG2_POINTS);
        const int nr_env = kKnobs.rrNr;
        const int nr = mode == GS_LINEAR && (nr_env == 2 || (nr_env == 0 && big)) ? 2 : 1;
        const bool wr = newtonish(mode) && !bconst;
        const int rr = 2 * nr + 1;
        const int rrows = rr * (wr ? 3 : 2) + 2;
        const size_t lds = sizeof(double) * ((size_t)RR2D_SLOTS * rrows * wxs * 2 * WAVE +
                                             (size_t)3 * (RR2D_WXMAX + 2) * rr * 2);
        const int64_t rows = (cl->ny + nr - 1) / nr;
        const void* fn = nullptr;
#define GS_RR2D_FN(M, N, U, W) fn = (const void*)&k_rr2d<M, N, U, W>
#define GS_RR2D_U(M, N, W) do { if (k.unit) GS_RR2D_FN(M, N, true, W); else GS_RR2D_FN(M, N, false, W); } while (0)
        if (mode == GS_LINEAR && nr == 2) GS_RR2D_U(GS_LINEAR, 2, false);
        else if (mode == GS_LINEAR) GS_RR2D_U(GS_LINEAR, 1, false);
        else if (mode == GS_NEWTON_B && wr) GS_RR2D_U(GS_NEWTON_B, 1, true);
        else if (mode == GS_NEWTON_B) GS_RR2D_U(GS_NEWTON_B, 1, false);
        else if (mode == GS_NONLINEAR) GS_RR2D_U(GS_NONLINEAR, 1, false);
        else GS_RR2D_U(GS_NEWTON, 1, true);
#undef GS_RR2D_U
#undef GS_RR2D_FN
        static std::mutex m;
        static std::map<std::pair<const void*, size_t>, int64_t> cap;
        int64_t resident = 0;
        {
            std::lock_guard<std::mutex> lk(m);
            const auto key = std::make_pair(fn, lds);
            auto it = cap.find(key);
            if (it == cap.end()) {
                int per = 0;
                if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess ||
                    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, (int)(WAVE * wxs), lds) != hipSuccess)
                    per = 0;
                (void)hipGetLastError();
                it = cap.emplace(key, per * device_cus()).first;
            }
            resident = it->second;
        }
        if (resident > 0) {
            // one round of resident blocks: z-chunks so that rows x chunks ~ the blocks the GPU holds at once
            const int64_t chunks = std::max<int64_t>(1, resident / rows);
            int64_t zc = (cl->nz + chunks - 1) / chunks;
            zc = zc < 1 ? 1 : zc;
            if (kKnobs.rrZcBig > 0 && big) zc = kKnobs.rrZcBig;
            if (kKnobs.rrZc > 0 && !big) zc = kKnobs.rrZc;
            const dim3 g((unsigned)rows, (unsigned)((cl->nz + zc - 1) / zc)), b(WAVE, (unsigned)wxs);
            Coef ka = k;
            const double *va = v, *fa = f, *wa = w;
            double *caa = ca, *cba = cb;
            int fnx = (int)fl->nx, fny = (int)fl->ny, fnz = (int)fl->nz, cnx = (int)cl->nx, cny = (int)cl->ny,
                cnz = (int)cl->nz, zca = (int)zc, zha = zhi ? 1 : 0;
            int64_t fldy = fl->ldy, fldz = fl->ldz, cldy = cl->ldy, cldz = cl->ldz;
            void* args[] = {&ka, &va, &fa, &wa, &caa, &cba, &fnx, &fny, &fnz, &fldy, &fldz,
                            &cnx, &cny, &cnz, &cldy, &cldz, &zca, &zha};
            const hipError_t e = hipLaunchKernel(fn, g, b, args, lds, st);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                return (int)e;
            }
            return launch_status();
        }
    }
    if (rr2) {
        // >= 2048 blocks of one coarse row where the level has them (chunks of <= 32 coarse planes)
        // LINEAR levels of >= 2^26 points: two coarse rows per block (231 VGPRs, 2 waves per SIMD): 0.507 vs
        // 0.529 ms at 512^3, but 0.072 vs 0.068 ms at 256^3 (gpurun_out/rrnr2, tools/rr_ab.py);
        // NONLINEAR / NEWTON: one row (VGPR budget). GS_RR_NR=1|2 forces the choice (A/B, tests).
        const int nr_env = kKnobs.rrNr;
        const bool big = fl->nx * fl->ny * fl->nz >= ((int64_t)1 << RR2_NR2_LOG2_POINTS);
        // (NEWTON with two rows spills 19 VGPRs: 40.5 vs 38.9 ms per 512^3 Newton iteration, gpurun_out/rrn)
        const int nr = mode == GS_LINEAR && (nr_env == 2 || (nr_env == 0 && big)) ? 2 : 1;
        // groups of coarse rows per block (k_rr2 NG; GS_RR_NG=2 where the rows fit twice in a block, A/B): two
        // y-neighbour rows in one 8-wave block cut the 512^3 launch's PMC reads from 1.139 to 1.089 x algorithmic
        // (NEWTON 1.157 -> 1.087) but run slower — k_rr2 0.479-0.512 vs 0.406-0.453 ms, V-cycle 2.111 vs
        // 2.055-2.065 ms, Newton 33.4-33.9 vs 32.8-33.4 ms (r05b, interleaved): two 4-wave blocks per CU at their
        // own barrier phases hide more latency than the halo rows the shared block saves; default one group
        const int ng = (kKnobs.rrNg == 2 && 2 * wxs <= RR2_WXMAX) ? 2 : 1;
        const int64_t rows = (cl->ny + nr * ng - 1) / (nr * ng); // blocks along y
        const int64_t chunks = (2048 + rows - 1) / rows;
        int64_t zc = (cl->nz + chunks - 1) / chunks;
        zc = zc < 1 ? 1 : (zc > 32 ? 32 : zc);
        // levels of >= 2^26 points: 64-coarse-plane chunks (512^3: 512 blocks, one round at two per CU): k_rr2
        // 0.454-0.462 vs 0.496-0.500 ms, V-cycle 2.111-2.118 vs 2.145-2.148 ms; 1024^3: 4.06 vs 4.12 ms,
        // V-cycle 16.71 vs 16.83-16.86 ms (16 / 32 / 128 planes all slower; profiles/r04/r04w_rr2_zc_big_ab.txt)
        if (big) zc = cl->nz < 64 ? (cl->nz < 1 ? 1 : cl->nz) : 64;
        if (kKnobs.rrZc > 0 && !big) zc = kKnobs.rrZc;       // (A/B: fine levels of < 2^26 points)
        if (kKnobs.rrZcBig > 0 && big) zc = kKnobs.rrZcBig; // (A/B: fine levels of >= 2^26 points)
        const dim3 g((unsigned)rows, (unsigned)((cl->nz + zc - 1) / zc)), b(WAVE, (unsigned)wxs, (unsigned)ng);
        // one operand slot (154 VGPRs, 3 waves per SIMD) measured 1.5 % (level 0) to 9 % (level 1) faster
        // than the two-slot prefetch ring (228 VGPRs, 2 waves per SIMD): tools/ab_session.sh, ab5
        // two-row blocks: the rows no neighbouring block reads are non-temporal loads (0.490 vs 0.505 ms at
        // 512^3, r02 tools/rr_ab_session.sh rrntu); since r05 one-row blocks too (their middle row's f and w: NEWTON_B
        // level 0 and the LINEAR levels below 2^26 points; Newton iteration 27.73-27.76 vs 27.86-27.97 ms, V-cycle
        // 2.097-2.100 vs 2.101-2.108 ms, r05w); GS_RR_NTU=0 keeps them cached, =1 restores the two-row-only rule (A/B)
        const int ntu_env = kKnobs.rrNtu;
        const bool ntu = ntu_env == 2 || (ntu_env == 1 && nr == 2);
#define GS_RR2G(M, N, U, T, G) hipLaunchKernelGGL((k_rr2<M, false, N, U, T, G>), g, b, 0, st, k, v, f, w, ca, cb, (int)fl->nx, (int)fl->ny, (int)fl->nz, fl->ldy, fl->ldz, (int)cl->nx, (int)cl->ny, (int)cl->nz, cl->ldy, cl->ldz, (int)zc, zhi ? 1 : 0, kKnobs.rrReverse)
#define GS_RR2V(M, N, U, T) do { if (ng == 2) GS_RR2G(M, N, U, T, 2); else GS_RR2G(M, N, U, T, 1); } while (0)
#define GS_RR2U(M, N, U) do { if (ntu) GS_RR2V(M, N, U, true); else GS_RR2V(M, N, U, false); } while (0)
#define GS_RR2(M, N) do { if (k.unit) GS_RR2U(M, N, true); else GS_RR2U(M, N, false); } while (0)
        if (mode == GS_LINEAR && nr == 2) GS_RR2(GS_LINEAR, 2);
        else if (mode == GS_LINEAR) GS_RR2(GS_LINEAR, 1);
        else if (mode == GS_NONLINEAR) GS_RR2(GS_NONLINEAR, 1);
        else if (mode == GS_NEWTON_B) GS_RR2(GS_NEWTON_B, 1);
        else GS_RR2(GS_NEWTON, 1);
#undef GS_RR2
#undef GS_RR2U
#undef GS_RR2V
#undef GS_RR2G
        return launch_status();
    }
    StencilOffsets so;
    for (int t = 0; t < 7; t++) {
        so.lds[t] = S->ox[t] + S->oy[t] * RR_VX;
        so.oz[t] = S->oz[t];
    }
    const int64_t tiles = ((cl->nx + RR_TXC - 1) / RR_TXC) * ((cl->ny + RR_TYC - 1) / RR_TYC);
    int64_t zc = tiles * cl->nz / 4096; // >= 4096 blocks where the level has them, 1..16 planes each
    zc = zc < 1 ? 1 : (zc > 16 ? 16 : zc);
    const dim3 g((unsigned)((cl->nx + RR_TXC - 1) / RR_TXC), (unsigned)((cl->ny + RR_TYC - 1) / RR_TYC),
                 (unsigned)((cl->nz + zc - 1) / zc));
#define GS_RR(M) hipLaunchKernelGGL(k_resrestrict<M>, g, dim3(RR_T), 0, st, k, so, v, f, w, ca, cb, (int)fl->nx, (int)fl->ny, (int)fl->nz, fl->ldy, fl->ldz, (int)cl->nx, (int)cl->ny, (int)cl->nz, cl->ldy, cl->ldz, (int)zoff, (int)zc)
    if (mode == GS_LINEAR) GS_RR(GS_LINEAR);
    else if (mode == GS_NONLINEAR) GS_RR(GS_NONLINEAR);
    else if (mode == GS_NEWTON_B) GS_RR(GS_NEWTON_B);
    else GS_RR(GS_NEWTON);
#undef GS_RR
    return launch_status();
}

int gs_restrict(const double* fine, const gs_level* fl, double* coarse, const gs_level* cl, hipStream_t st)
{
    return gs_restrict2(fine, fl, coarse, nullptr, cl, st);
}

int gs_interpolate(const double* coarse, const gs_level* cl, double* e, const gs_level* fl, hipStream_t st)
{
    if (!coarse || !e || bad_level(fl) || bad_level(cl) || fl->z0 != 0 || cl->z0 != 0) return GS_EINVAL;
    if ((fl->nx + 1) / 2 > cl->nx + 1 || (fl->ny + 1) / 2 > cl->ny + 1 || (fl->nz + 1) / 2 > cl->nz + 1) return GS_EINVAL;
    const dim3 g((unsigned)((fl->nx + 2 + 63) / 64), (unsigned)((fl->ny + 2 + 3) / 4), (unsigned)(fl->nz + 2)), b(64, 4);
    hipLaunchKernelGGL(k_interpolate, g, b, 0, st, coarse, e, (int)fl->nx + 2, (int)fl->ny + 2, (int)fl->nz + 2,
                       fl->ldy, fl->ldz, cl->ldy, cl->ldz);
    return launch_status();
}

int gs_prolong_add(const double* coarse_v, const double* coarse_sub, const gs_level* cl, double* fine_v,
                   const gs_level* fl, hipStream_t st)
{
    if (!coarse_v || !fine_v || bad_level(fl) || bad_level(cl)) return GS_EINVAL;
    if (fl->nx == 0 || fl->ny == 0 || fl->nz == 0) return 0;
    // coarse planes read: global floor(gz/2) and +1 for fine global gz in [fz0+1, fz0+fnz]
    const int64_t clo = (fl->z0 + 1) / 2 - cl->z0, chi = (fl->z0 + fl->nz) / 2 + 1 - cl->z0;
    if ((fl->nx + 1) / 2 > cl->nx + 1 || (fl->ny + 1) / 2 > cl->ny + 1 || clo < 0 || chi > cl->nz + 1)
        return GS_EINVAL;
    const dim3 g((unsigned)((fl->nx + 127) / 128), (unsigned)((fl->ny + 3) / 4), (unsigned)fl->nz), b(64, 4);
    if (coarse_sub)
        hipLaunchKernelGGL(k_prolong_add<true>, g, b, 0, st, coarse_v, coarse_sub, fine_v, (int)fl->nx, (int)fl->ny,
                           (int)fl->nz, fl->ldy, fl->ldz, cl->ldy, cl->ldz, (int)fl->z0, (int)cl->z0);
    else
        hipLaunchKernelGGL(k_prolong_add<false>, g, b, 0, st, coarse_v, nullptr, fine_v, (int)fl->nx, (int)fl->ny,
                           (int)fl->nz, fl->ldy, fl->ldz, cl->ldy, cl->ldz, (int)fl->z0, (int)cl->z0);
    return launch_status();
}

int gs_apply_op(const gs_stencil* S, const gs_level* L, double gamma, const double* u, double* out, hipStream_t st)
{
    if (!out) return GS_EINVAL;
    return launch_pass<2, false>(S, L, GS_NONLINEAR, 0.0, gamma, u, nullptr, nullptr, out, nullptr, st);
}

int gs_apply_op_add(const gs_stencil* S, const gs_level* L, double gamma, const double* u, double* f, hipStream_t st)
{
    if (!f) return GS_EINVAL;
    return launch_pass<2, true>(S, L, GS_NONLINEAR, 0.0, gamma, u, nullptr, nullptr, f, nullptr, st);
}

int gs_newton_F(const gs_stencil* S, const gs_level* L, double gamma, const double* w, const double* F, double* f,
                double* partials, hipStream_t st)
{
    if (!f || !F) return GS_EINVAL;
    // compF (NewtonSolver.cpp:48-81) is the NONLINEAR residual of newtonV against newtonF
    return gs_residual(S, L, GS_NONLINEAR, gamma, w, F, nullptr, f, partials, st);
}

int gs_newton_F_update_supported(const gs_stencil* S, const gs_level* L)
{
    return (S && !bad_level(L) && valid_stencil(S) && L->nx > 0 && L->ny > 0 && L->nz > 0 && pass_plan(S, L).rb) ? 1
                                                                                                               : 0;
}

int gs_newton_F_update(const gs_stencil* S, const gs_level* L, double gamma, const double* w, const double* e,
                       const double* F, double* w_out, double* f, double* partials, hipStream_t st)
{
    if (!w || !e || !F || !w_out || !f || w_out == w || w_out == e || !gs_newton_F_update_supported(S, L))
        return GS_EINVAL;
    const Coef k = make_coef(S, L, 0.0, gamma);
    const PassPlan plan = pass_plan(S, L); // the grid and partial layout of gs_newton_F (k_rb KIND 1)
    const dim3 b(WAVE, RB_W);
    if (k.unit)
        hipLaunchKernelGGL((k_newton_upd<RB_RY, RB_W, true>), plan.grid, b, 0, st, k, w, e, F, w_out, f, partials,
                           (int)L->nx, (int)L->ny, (int)L->nz, L->ldy, L->ldz, plan.zc, nullptr, 0, 0, 0, 0, 0, nullptr);
    else
        hipLaunchKernelGGL((k_newton_upd<RB_RY, RB_W, false>), plan.grid, b, 0, st, k, w, e, F, w_out, f, partials,
                           (int)L->nx, (int)L->ny, (int)L->nz, L->ldy, L->ldz, plan.zc, nullptr, 0, 0, 0, 0, 0, nullptr);
    return launch_status();
}

int gs_newton_F_update_restrict_supported(const gs_stencil* S, const gs_level* L, const gs_level* cl)
{
    // a whole level (z0 = 0) and its coarse level (n/2 per axis, the hierarchy's), RB_RY = 2 rows per wave
    return (gs_newton_F_update_supported(S, L) && cl && !bad_level(cl) && L->z0 == 0 && cl->z0 == 0 &&
            cl->nx == L->nx / 2 && cl->ny == L->ny / 2 && cl->nz == L->nz / 2 && cl->nx > 0 && cl->ny > 0 && cl->nz > 0)
               ? 1
               : 0;
}

int gs_newton_F_update_restrict(const gs_stencil* S, const gs_level* L, double gamma, const double* w, const double* e,
                                const double* F, double* w_out, double* f, double* partials, double* coarse_w,
                                const gs_level* cl, hipStream_t st)
{
    return gs_newton_F_update_restrict_bfac(S, L, gamma, w, e, F, w_out, f, partials, coarse_w, cl, nullptr, st);
}

int gs_newton_F_update_restrict_bfac(const gs_stencil* S, const gs_level* L, double gamma, const double* w,
                                     const double* e, const double* F, double* w_out, double* f, double* partials,
                                     double* coarse_w, const gs_level* cl, double* b_out, hipStream_t st)
{
    if (!w || !e || !F || !w_out || !f || !coarse_w || w_out == w || w_out == e ||
        (b_out && (b_out == w_out || b_out == w || b_out == e || b_out == f)) ||
        !gs_newton_F_update_restrict_supported(S, L, cl))
        return GS_EINVAL;
    static_assert(RB_RY == 2, "the fused restriction takes two fine rows per wave");
    const Coef k = make_coef(S, L, 0.0, gamma);
    const PassPlan plan = pass_plan(S, L); // the same grid / partials as gs_newton_F_update
    const dim3 b(WAVE, RB_W);
#define GS_NUR(U, B) hipLaunchKernelGGL((k_newton_upd<RB_RY, RB_W, U, true, B>), plan.grid, b, 0, st, k, w, e, F, w_out, f, partials, (int)L->nx, (int)L->ny, (int)L->nz, L->ldy, L->ldz, plan.zc, coarse_w, (int)cl->nx, (int)cl->ny, (int)cl->nz, cl->ldy, cl->ldz, b_out)
    if (b_out) {
        if (k.unit) GS_NUR(true, true);
        else GS_NUR(false, true);
    } else {
        if (k.unit) GS_NUR(true, false);
        else GS_NUR(false, false);
    }
#undef GS_NUR
    return launch_status();
}

int gs_newton_bfac(const gs_level* L, double gamma, const double* w, double* b, hipStream_t st)
{
    if (bad_level(L) || !w || !b) return GS_EINVAL;
    const int64_t n = L->ldz * (L->nz + 4); // planes -1 .. nz+2
    const double *ws = w - L->ldz;
    double* bs = b - L->ldz;
    if (ws < bs + n && bs < ws + n) return GS_EINVAL;
    const uintptr_t a = reinterpret_cast<uintptr_t>(bs), c = reinterpret_cast<uintptr_t>(ws);
    if ((a & 7) || (c & 7)) return GS_EINVAL;
    const int head = ((a ^ c) & 15) ? -1 : (int)((a & 15) / 8); // -1: no common dwordx4 alignment
    hipLaunchKernelGGL(k_bfac, dim3(1024), dim3(256), 0, st, bs, ws, n, gamma, head);
    return launch_status();
}

int gs_fill(double* dst, double value, int64_t n, hipStream_t st)
{
    if (!dst || n < 0) return GS_EINVAL;
    if (n == 0) return 0;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_fill, dim3((unsigned)blocks), dim3(256), 0, st, dst, value, n);
    return launch_status();
}

int gs_copy(double* dst, const double* src, int64_t n, hipStream_t st)
{
    if (!dst || !src || n < 0) return GS_EINVAL;
    if (n == 0 || dst == src) return 0;
    const uintptr_t a = reinterpret_cast<uintptr_t>(dst), b = reinterpret_cast<uintptr_t>(src);
    if (((a ^ b) & 15) || (a & 7)) // no common dwordx4 alignment
        return (int)hipMemcpyAsync(dst, src, sizeof(double) * n, hipMemcpyDeviceToDevice, st);
    hipLaunchKernelGGL(k_copy, dim3(1024), dim3(256), 0, st, dst, src, n, (a & 15) ? 1 : 0);
    return launch_status();
}

int gs_axpy(double* y, const double* x, double a, int64_t n, hipStream_t st)
{
    if (!y || !x || n < 0) return GS_EINVAL;
    if (n == 0) return 0;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_axpy, dim3((unsigned)blocks), dim3(256), 0, st, y, x, a, n);
    return launch_status();
}

int gs_coarse_cycle_max_levels(void) { return CC_MAXLEV; }

int gs_coarse_cycle(const gs_stencil* S, const gs_coarse_level* lv, int n, int mode, double omega, double gamma,
                    int pre, int post, hipStream_t st)
{
    mode = base_mode(mode); // (the coarse levels read their factor fields, which hold gamma under GS_NEWTON_G)
    if (!S || !valid_stencil(S) || !lv || n < 1 || n > CC_MAXLEV || mode < GS_LINEAR || mode > GS_NEWTON_B ||
        pre < 0 || post < 0)
        return GS_EINVAL;
    CcPlan P{};
    P.n = n;
    P.pre = pre;
    P.post = post;
    for (int l = 0; l < n; l++) {
        const gs_coarse_level& a = lv[l];
        const gs_level* g = &a.geom;
        if (bad_level(g) || g->z0 != 0 || g->nx < 1 || g->ny < 1 || g->nz < 1 ||
            g->nx * g->ny * g->nz > (int64_t)INT32_MAX || !a.v || !a.v_alt || a.v == a.v_alt || !a.f ||
            (l + 1 < n && !a.r) || (newtonish(mode) && !a.newton_v) ||
            (mode == GS_NONLINEAR && ((l > 0 && !a.rest_v) || a.v_zero)))
            return GS_EINVAL;
        if (l > 0) { // consecutive levels of one hierarchy (the restriction / prolongation bounds)
            const gs_level* fg = &lv[l - 1].geom;
            if (g->nx != fg->nx / 2 || g->ny != fg->ny / 2 || g->nz != fg->nz / 2) return GS_EINVAL;
        }
        CcLevel& L = P.L[l];
        L.v = a.v;
        L.va = a.v_alt;
        L.f = a.f;
        L.r = a.r;
        L.rv = a.rest_v;
        L.w = a.newton_v;
        L.ldy = g->ldy;
        L.ldz = g->ldz;
        L.nx = (int)g->nx;
        L.ny = (int)g->ny;
        L.nz = (int)g->nz;
        L.vz = a.v_zero != 0;
        L.k = make_coef(S, g, omega, gamma);
    }
    if (mode == GS_LINEAR) hipLaunchKernelGGL(k_coarse_cycle<GS_LINEAR>, dim3(1), dim3(CC_T), 0, st, P);
    else if (mode == GS_NONLINEAR) hipLaunchKernelGGL(k_coarse_cycle<GS_NONLINEAR>, dim3(1), dim3(CC_T), 0, st, P);
    else if (mode == GS_NEWTON_B) hipLaunchKernelGGL(k_coarse_cycle<GS_NEWTON_B>, dim3(1), dim3(CC_T), 0, st, P);
    else hipLaunchKernelGGL(k_coarse_cycle<GS_NEWTON>, dim3(1), dim3(CC_T), 0, st, P);
    return launch_status();
}

const char* gs_strerror(int code)
{
    if (code == 0) return "success";
    if (code == GS_EINVAL) return "gpusolve: invalid argument";
    return hipGetErrorString((hipError_t)code);
}

const char* gs_build_info(void)
{
    return "gpusolve_hip v13: pairs k_tb2y(4x2 waves, 2 rows/wave, one round of z-chunks on large levels, LINEAR 2-step prefetch; +prolong; "
           "512-point column blocks for longer rows in every mode; from 64^3 levels; zero-iterate chunks fitted to "
           "resident rounds; zero iterates q = +0; whole-wave rows without range selects (FX); LINEAR loads grouped by "
           "field; x-edge values in VGPRs for LINEAR and the NEWTON_B whole-row plain pair), sweeps k_rb(ry2 w4 zc<=32 "
           "dpp nt), fused residual+restriction (2 coarse rows per block from 2^26 points, descending z-chunks, halo rows "
           "loaded first, non-temporal unshared rows), NEWTON update + "
           "compF (+ level-1 restriction, + the next factor B), NEWTON inner solves on B (GS_NEWTON_B: reciprocal "
           "quotient, shared per pair; GS_NEWTON_G: B = gamma unread), unit-neighbour stencil sums, tiled small levels, "
           "one-workgroup coarse cycle; fp-contract=off";
}

} // extern "C"

#ifdef GS_EXP_EFIELD
// timing-only build (gs_device.hpp): the E field's element distance from newtonV
extern "C" void gs_exp_set_efoff(int64_t n) { gs_exp_efoff = n; }
#endif
