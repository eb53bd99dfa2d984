// gs_diag.hip — libgpusolve_diag.so (include/gpusolve_diag.h): measurement and tuning code that is NOT
// part of the product: the tuning variants of the sweep and pair kernels (tools/kbench.py), streaming
// bandwidth probes (bench.py's measured ceiling, tools/), the exact-division check, and k_prr — the
// pre-smoothing pair + residual + restriction in one pass, built, bit-identical and measured slower than
// the two passes the driver runs, kept as a tested operator. Only tools/, tests/ and
// bench.py's measured-ceiling leg load this library.
#include "gs_device.hpp"
#include "gpusolve_diag.h"

namespace {

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
    if (n < 0 || (n & 1) || kind < 0 || kind > 4 || blocks <= 0) return GS_EINVAL;
    if (kind == 4) { // copy at RCCL's transport-kernel footprint (k_fatcopy)
        hipLaunchKernelGGL(k_fatcopy, dim3(blocks), dim3(256), 0, st, out, a, n / 2);
        return launch_status();
    }
    using K = void (*)(double*, const double*, const double*, int64_t, double*);
    static const K tab[4][2][2] = {
        {{k_bw<0, 1, false>, k_bw<0, 1, true>}, {k_bw<0, 4, false>, k_bw<0, 4, true>}},
        {{k_bw<1, 1, false>, k_bw<1, 1, true>}, {k_bw<1, 4, false>, k_bw<1, 4, true>}},
        {{k_bw<2, 1, false>, k_bw<2, 1, true>}, {k_bw<2, 4, false>, k_bw<2, 4, true>}},
        {{k_bw<3, 1, false>, k_bw<3, 1, true>}, {k_bw<3, 4, false>, k_bw<3, 4, true>}},
    };
    hipLaunchKernelGGL(tab[kind][unroll > 1][nt != 0], dim3(blocks), dim3(256), 0, st, out, a, b, n / 2, sink);
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

int gs_debug_stream_triad(double* out, const double* a, const double* b, int64_t n, hipStream_t st)
{
    if (!out || !a || !b || n < 0 || (n & 1)) return GS_EINVAL;
    hipLaunchKernelGGL(k_triad, dim3(4096), dim3(256), 0, st, out, a, b, n / 2);
    return launch_status();
}

} // extern "C"
