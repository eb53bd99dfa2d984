/* gpusolve_hip.h — the thin C-ABI launcher of the MI355X GMG V-cycle kernels (libgpusolve_hip.so).
 *
 * Every entry point replaces one operator of the reference CPU backend (Bricktricker/gpu-solve,
 * snapshot 2025-02-27; paths relative to that repository):
 *
 *   gs_rhs_init          CpuGridData ctor RHS fill            src/cpu/CpuGridData.cpp:44-78
 *   gs_jacobi_sweep      CpuSolver::jacobi (one sweep)         src/cpu/CpuSolver.cpp:141-180
 *   gs_residual          CpuSolver::compResidual (+ l2 norm)   src/cpu/CpuSolver.cpp:45-83
 *   gs_sumsq_finish      the sqrt(sum r^2) of compResidual     src/cpu/CpuSolver.cpp:51,77,82
 *   gs_restrict          CpuSolver::restrict                   src/cpu/CpuSolver.cpp:211-238
 *   gs_restrict2         two restrict calls of the FAS branch  src/cpu/CpuSolver.cpp:104-107
 *   gs_residual_restrict compResidual + restrict (r never stored) src/cpu/CpuSolver.cpp:98-99
 *   gs_jacobi_sweep2     two CpuSolver::jacobi sweeps fused    src/cpu/CpuSolver.cpp:141-180 (k=2)
 *   gs_interpolate       CpuSolver::interpolate                src/cpu/CpuSolver.cpp:240-290
 *   gs_prolong_add       interpolate + (v_c -= restV_c) + (v_f += e_f)
 *                                                              src/cpu/CpuSolver.cpp:121-132
 *   gs_apply_op          CpuSolver::applyStencil               src/cpu/CpuSolver.cpp:182-208
 *   gs_apply_op_add      applyStencil then f += r (FAS)        src/cpu/CpuSolver.cpp:110-112
 *   gs_newton_F          NewtonSolver::compF                   src/cpu/NewtonSolver.cpp:48-81
 *   gs_newton_F_update   findError's newtonV += v, then compF  src/cpu/NewtonSolver.cpp:105-107, 48-81
 *   gs_copy              Vector3 copy-assignment (newtonF = f) src/cpu/NewtonSolver.cpp:12
 *   gs_axpy              Vector3::operator+= / -=              src/cpu/Vector3.cpp:34-53
 *   gs_coarse_cycle      CpuSolver::vcycle below a level (one launch) src/cpu/CpuSolver.cpp:92-135
 *
 * Conventions
 *  - fp64 everywhere. A field of level (nx,ny,nz) is padded to (nx+2, ny+2, nz+2); element
 *    (x,y,z), 0 <= x <= nx+1 etc., lives at ptr[x + y*ldy + z*ldz]  (x unit-stride, z slowest;
 *    the reference's (x,y,z) semantics, not its z-fastest storage). `ptr` is the address of
 *    padded element (0,0,0). gs_field_layout() gives the pitches and an allocation recipe that
 *    makes every interior x=1 element 128-byte aligned (speed only; any pitch >= nx+2 is correct)
 *    and provides planes z = -1 and z = nz+2 (the second ghost plane of a Z-slab, read only by the
 *    fused two-sweep launcher gs_jacobi_sweep2 when a slab side is an internal boundary).
 *  - Stencil: 7 (value, offset) pairs in config order, offsets in {-1,0,1}. The canonical order
 *    (centre, +x, -x, +y, -y, +z, -z) of every reference config runs the LDS/register-tiled fast
 *    kernels; any other order or shape runs a generic kernel. Sums are evaluated in config order.
 *  - Launchers are asynchronous on `stream`, never allocate, never synchronise, are reentrant.
 *    Scratch (residual partials) is caller-owned. Return 0 on success, else a hipError_t value
 *    (or GS_EINVAL) — see gs_strerror().
 *  - Boundary (padding) values of v / e / r / restV are never written and must hold 0, as on
 *    every reference path.
 */
#ifndef GPUSOLVE_HIP_H
#define GPUSOLVE_HIP_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_EINVAL 100001 /* bad argument (shape, stencil offset outside {-1,0,1}, null pointer) */

enum { GS_LINEAR = 0, GS_NONLINEAR = 1, GS_NEWTON = 2 }; /* GridParams::Mode, src/gridParams.h:29-33 */
/* Not a reference mode (added): NEWTON's linearised operator with the point's linearisation factor precomputed.
 * Every launcher that takes `mode` and a `w` operand accepts it; `w` then holds B = gamma*(1+newtonV)*exp(newtonV)
 * (gs_newton_bfac) instead of newtonV. The Jacobi denominator preFac + B is bit for bit the reference's
 * preFac + gamma*(1+w)*exp(w) (CpuSolver.cpp:166-172); the operator term is B*v instead of the reference's
 * (gamma*(1+w)*v)*exp(w) (CpuSolver.cpp:63-66), one product re-associated (a rounding of the term, like glibc's
 * vs ocml's exp). The host driver's inner Newton solves run in this mode: exp(newtonV) is evaluated once per
 * point and Newton iteration instead of in every sweep, residual and restriction of the ten inner V-cycles. */
enum { GS_NEWTON_B = 3 };
/* GS_NEWTON_B whose factor field holds gamma at every point, the first Newton iteration's B = gamma*(1+0)*exp(0)
 * (newtonV = 0). Accepted wherever GS_NEWTON_B is; `w` must still point at that field, filled with gamma (gs_fill).
 * The fused pairs (gs_jacobi_sweep2*, gs_jacobi_sweep2_prolong*) and the register residual + restriction
 * (gs_residual_restrict*, k_rr2) then take gamma instead of loading w (8 B per point less); every other launcher reads
 * the field. Same values as GS_NEWTON_B on that field, bit for bit. */
enum { GS_NEWTON_G = 4 };

/* GridParams::stencil (src/gridParams.h:7-27): values + (x,y,z) offsets, config order. */
typedef struct {
    double s[7];
    int ox[7], oy[7], oz[7];
} gs_stencil;

/* One level (or one Z-slab of a level) of the hierarchy. */
typedef struct {
    int64_t nx, ny, nz; /* interior extents of this level; for a slab nz is the local plane count */
    int64_t ldy, ldz;   /* element pitch of a y-row / a z-plane (ldy >= nx+2, ldz >= ldy*(ny+2)) */
    int64_t z0;         /* global index offset of local plane 0 (0 unless Z-slab partitioned)     */
    double h;           /* mesh width h_l = 1/(ny_l + 1)  (src/cpu/CpuGridData.cpp:41)              */
} gs_level;

/* Pitches and allocation recipe for a level with interior (nx,ny,nz): allocate alloc_elems
 * doubles 256-B aligned and use base + origin_offset as the field pointer. */
int gs_field_layout(int64_t nx, int64_t ny, int64_t nz, int64_t* ldy, int64_t* ldz, int64_t* alloc_elems,
                    int64_t* origin_offset);

/* Level-0 right-hand side (mode LINEAR: interior, x = (X-1)*h0; otherwise the whole padded
 * array, x = X*h0, with gamma). h0 = 1/(Y+1) (src/main.cpp:84). */
int gs_rhs_init(const gs_level* L, double* f, int mode, double h0, double gamma, hipStream_t stream);

/* One damped-Jacobi sweep, residual and update fused: v_out = v_in + omega * D^-1 (f - A v_in).
 * w = newtonV of this level (mode NEWTON), ignored otherwise. v_in and v_out must differ.
 * v_in = NULL: the zero iterate, not read (modes LINEAR / NEWTON; the coarse-level first sweep after
 * the reference's v = 0, CpuSolver.cpp:114-116) — bit-identical to passing a zeroed field. */
int gs_jacobi_sweep(const gs_stencil* S, const gs_level* L, int mode, double omega, double gamma,
                    const double* v_in, double* v_out, const double* f, const double* w, hipStream_t stream);

/* The same sweep, also writing the per-block sums of r^2 of the residual r = f - A(v_in) it computes
 * (the reference's compResidual norm of the pre-sweep iterate; layout as gs_residual's partials). */
int gs_jacobi_sweep_norm(const gs_stencil* S, const gs_level* L, int mode, double omega, double gamma,
                         const double* v_in, double* v_out, const double* f, const double* w, double* partials,
                         hipStream_t stream);

/* Two fused sweeps, v_out = S(S(v_in)), reading v_in / f once (temporal blocking; bit-identical to
 * two gs_jacobi_sweep calls; v_in = NULL: the zero iterate, as for gs_jacobi_sweep). gs_jacobi_sweep2_supported(S, L): 0 impossible (stencil not in
 * canonical order, or, in some mode, nx > 1024), 1 possible, 2 possible and large enough to fill the GPU
 * (the driver uses it only then). zlo / zhi: the plane below local plane 1
 * (resp. above plane nz) is an internal Z-slab boundary whose two ghost planes (0 and -1, resp.
 * nz+1 and nz+2) of v_in are current; 0 = a level boundary. The x-boundary columns (x = 0 and
 * nx+1) of v_in must be zero, as the reference's are (homogeneous Dirichlet, never written). */
int gs_jacobi_sweep2_supported(const gs_stencil* S, const gs_level* L);
/* The same for one mode (rows of more than 512 points: column blocks in LINEAR / NONLINEAR mode, any
 * row length; NEWTON up to 1024 points). gs_jacobi_sweep2_supported is the minimum over the modes. */
int gs_jacobi_sweep2_supported_mode(const gs_stencil* S, const gs_level* L, int mode);
int gs_jacobi_sweep2(const gs_stencil* S, const gs_level* L, int mode, double omega, double gamma,
                     const double* v_in, double* v_out, const double* f, const double* w, int zlo, int zhi,
                     hipStream_t stream);
/* The fused pair, also writing gs_jacobi_sweep2_num_partials(S, L, mode) per-block sums of r^2 of the
 * residual r = f - A(v_in) its first sweep computes (the compResidual norm of v_in, fixed order; the
 * block shape, hence the count, depends on the mode). */
int gs_jacobi_sweep2_norm(const gs_stencil* S, const gs_level* L, int mode, double omega, double gamma,
                          const double* v_in, double* v_out, const double* f, const double* w, int zlo, int zhi,
                          double* partials, hipStream_t stream);
int64_t gs_jacobi_sweep2_num_partials(const gs_stencil* S, const gs_level* L, int mode);
/* Prolongation + correction fused into the first post-smoothing pair: v_out = S(S(v_in + P(c))) with
 * c = coarse_v (LINEAR) or coarse_v - coarse_sub (NONLINEAR, FAS: CpuSolver.cpp:121-125), P the
 * trilinear interpolation of gs_prolong_add; bit-identical to gs_prolong_add followed by
 * gs_jacobi_sweep2, with the corrected iterate never stored. Replaces CpuSolver.cpp:127-135
 * (interpolate, v += e, jacobi(post)) for the first two post-smoothing sweeps. Supported
 * (gs_jacobi_sweep2_prolong_supported != 0) for LINEAR and NEWTON levels of rows <= 512 points, and
 * LINEAR and NEWTON levels of longer rows (with a workspace, gs_jacobi_sweep2_prolong_ws), whose z0 is even (a level, a Z-slab of one, or a plane range of either); coarse_sub must then be NULL. Fine local
 * plane z interpolates from coarse planes (z + z0) / 2 - coarse->z0 (+1); zlo / zhi as for
 * gs_jacobi_sweep2 — the ghost planes of an internal side are corrected too, from the coarse field's
 * planes under them (coarse ghost planes -1 / nz+1 must then be current). w: the level's newtonV
 * for a NEWTON level, else ignored. */
int gs_jacobi_sweep2_prolong_supported(const gs_stencil* S, const gs_level* L, int mode);
int gs_jacobi_sweep2_prolong(const gs_stencil* S, const gs_level* L, int mode, double omega, double gamma,
                             const double* v_in, const double* coarse_v, const double* coarse_sub,
                             const gs_level* coarse, double* v_out, const double* f, const double* w, int zlo,
                             int zhi, hipStream_t stream);
/* The same with a device workspace, which LINEAR levels of rows longer than 512 points (the column-block
 * pair: BASELINE config #5's 1024-point rows) need: gs_jacobi_sweep2_prolong_ws_elems doubles (0 when
 * none is needed; gs_jacobi_sweep2_prolong is this call with no workspace and fails with GS_EINVAL
 * where one is needed). The launch first writes the corrected iterate of the four columns around
 * every interior column-block boundary into it (the neighbouring blocks' edge columns), then runs the
 * pair; concurrent launches need separate workspaces. */
int64_t gs_jacobi_sweep2_prolong_ws_elems(const gs_stencil* S, const gs_level* L, int mode);
int gs_jacobi_sweep2_prolong_ws(const gs_stencil* S, const gs_level* L, int mode, double omega, double gamma,
                                const double* v_in, const double* coarse_v, const double* coarse_sub,
                                const gs_level* coarse, double* v_out, const double* f, const double* w, int zlo,
                                int zhi, double* ws, int64_t ws_elems, hipStream_t stream);
/* Small levels (LINEAR or NEWTON, canonical stencil order, whole levels: z0 = 0), where every operator
 * is launch latency: a level's down-leg step and up-leg step each in ONE launch of 8^3-point LDS tiles
 * that recompute their halos (no exchange between blocks), bit-identical to the unfused sequences.
 *   gs_smooth2_restrict_tiled  v_out = S(S(v_in)) (v_in NULL: v = 0), coarse_f = R(f - A v_out)
 *                              == two jacobi sweeps + compResidual + restrict     CpuSolver.cpp:88-99,141-180,211-238
 *                              (coarse = fine / 2 per axis)
 *   gs_prolong_smooth2_tiled   v_out = S(S(v_in + P coarse_v))
 *                              == interpolate + v += e + two jacobi sweeps        CpuSolver.cpp:127-134,240-290
 * w: the level's newtonV in NEWTON mode (else ignored). v_in and v_out are distinct fields of the level's
 * layout; only interior points of v_out are written. */
int gs_tiled_supported(const gs_stencil* S, const gs_level* L, int mode);
int gs_smooth2_restrict_tiled(const gs_stencil* S, const gs_level* fine, int mode, double omega, double gamma,
                              const double* v_in, double* v_out, const double* f, const double* w, double* coarse_f,
                              const gs_level* coarse, hipStream_t stream);
int gs_prolong_smooth2_tiled(const gs_stencil* S, const gs_level* fine, int mode, double omega, double gamma,
                             const double* v_in, const double* coarse_v, const gs_level* coarse, double* v_out,
                             const double* f, const double* w, hipStream_t stream);
/* Which fused-pair kernel (and shape) gs_jacobi_sweep2 launches for this level and mode ("" if none). */
const char* gs_jacobi_sweep2_kernel(const gs_stencil* S, const gs_level* L, int mode);

/* r = f - A(v) on the interior. r may be NULL (norm only). partials may be NULL (no norm);
 * otherwise it receives gs_residual_num_partials(S, L) per-block sums of r^2 in a fixed order. */
int gs_residual(const gs_stencil* S, const gs_level* L, int mode, double gamma, const double* v, const double* f,
                const double* w, double* r, double* partials, hipStream_t stream);
int64_t gs_residual_num_partials(const gs_stencil* S, const gs_level* L);

/* *out = sqrt(sum partials[0..n)) summed in a fixed order (deterministic). If accumulate is
 * non-zero the square root is skipped and the sum is written (for cross-slab reductions). */
int gs_sumsq_finish(const double* partials, int64_t n, double* out, int accumulate, hipStream_t stream);

/* 27-point full weighting of fine onto the coarse interior. */
/* Fused residual + full weighting: coarse = R(f - A(v)) on the coarse interior, with the fine
 * residual never stored (bit-identical to gs_residual followed by gs_restrict2). cb may be NULL.
 * Replaces src/cpu/CpuSolver.cpp:45-83 + :211-238 as called at CpuSolver.cpp:98-99. */
int gs_residual_restrict(const gs_stencil* S, const gs_level* fine, int mode, double gamma, const double* v,
                         const double* f, const double* w, double* coarse_a, double* coarse_b,
                         const gs_level* coarse, hipStream_t stream);
/* The same on a Z-slab whose top (plane fine->nz + 1) is an internal boundary when zhi != 0: the
 * residual on that ghost plane is evaluated from the current ghost planes nz+1 of v, f, w and nz+2
 * of v instead of being the zero of a level boundary. Coarse plane z must sit over fine plane 2z
 * (2 coarse->z0 == fine->z0), canonical stencil, rows <= 1024 points
 * (gs_residual_restrict_slab_supported(S, fine) != 0 and the plane condition); GS_EINVAL otherwise. */
int gs_residual_restrict_slab_supported(const gs_stencil* S, const gs_level* fine);
int gs_residual_restrict_slab(const gs_stencil* S, const gs_level* fine, int mode, double gamma, const double* v,
                              const double* f, const double* w, double* coarse_a, double* coarse_b,
                              const gs_level* coarse, int zhi, hipStream_t stream);
int gs_restrict(const double* fine, const gs_level* fl, double* coarse, const gs_level* cl, hipStream_t stream);
/* Same, writing two coarse outputs (FAS restV and v). */
int gs_restrict2(const double* fine, const gs_level* fl, double* coarse_a, double* coarse_b, const gs_level* cl,
                 hipStream_t stream);

/* Trilinear prolongation of the coarse field into the fine e (whole padded fine array; index
 * P-1 of each axis is written 0). */
int gs_interpolate(const double* coarse, const gs_level* cl, double* e, const gs_level* fl, hipStream_t stream);

/* Fused correction: fine_v(interior) += P(coarse_v - coarse_sub) (coarse_sub may be NULL). */
int gs_prolong_add(const double* coarse_v, const double* coarse_sub, const gs_level* cl, double* fine_v,
                   const gs_level* fl, hipStream_t stream);

/* out = A(u)/h^2 + gamma*u*exp(u) on the interior (FAS coarse operator). */
int gs_apply_op(const gs_stencil* S, const gs_level* L, double gamma, const double* u, double* out,
                hipStream_t stream);
/* f += A(u)/h^2 + gamma*u*exp(u) on the interior. */
int gs_apply_op_add(const gs_stencil* S, const gs_level* L, double gamma, const double* u, double* f,
                    hipStream_t stream);

/* Newton outer residual f = F - [A(w)/h^2 + gamma*w*exp(w)] (+ partial sums of f^2 as gs_residual). */
int gs_newton_F(const gs_stencil* S, const gs_level* L, double gamma, const double* w, const double* F, double* f,
                double* partials, hipStream_t stream);

/* findError's newtonV += v followed by compF (NewtonSolver.cpp:105-107, then :48-81) in one pass:
 * w_out = w + e at every interior point and f = F - [A(w_out)/h^2 + gamma*w_out*exp(w_out)] (+ the
 * partial sums of f^2 of gs_newton_F, same count and order), bit-identical to gs_axpy(w, e, 1) then
 * gs_newton_F. w_out must be a third field whose non-interior cells already hold w + e there (zeros
 * on a whole level, the Dirichlet boundary). Shapes without the register-blocked pass (tiny levels,
 * non-canonical stencils): _supported() == 0 and EINVAL. */
int gs_newton_F_update_supported(const gs_stencil* S, const gs_level* L);
int gs_newton_F_update(const gs_stencil* S, const gs_level* L, double gamma, const double* w, const double* e,
                       const double* F, double* w_out, double* f, double* partials, hipStream_t stream);
/* The same pass plus findError's restriction of the new newtonV onto the next level (NewtonSolver.cpp:88-92):
 * coarse_w (the coarse level's newtonV, interior written) = R(w_out), bit-identical to gs_restrict(w_out, ...)
 * after gs_newton_F_update; whole levels (z0 = 0) whose coarse level has n/2 points per axis. */
int gs_newton_F_update_restrict_supported(const gs_stencil* S, const gs_level* L, const gs_level* coarse);
int gs_newton_F_update_restrict(const gs_stencil* S, const gs_level* L, double gamma, const double* w, const double* e,
                                const double* F, double* w_out, double* f, double* partials, double* coarse_w,
                                const gs_level* coarse, hipStream_t stream);
/* The same pass plus the next inner solve's GS_NEWTON_B factor of this level (added): b_out = bfac(w_out) at the
 * interior points — gs_newton_bfac's values there, from the exp(w_out) compF evaluates anyway. NULL: exactly the
 * call above. */
int gs_newton_F_update_restrict_bfac(const gs_stencil* S, const gs_level* L, double gamma, const double* w,
                                     const double* e, const double* F, double* w_out, double* f, double* partials,
                                     double* coarse_w, const gs_level* coarse, double* b_out, hipStream_t stream);

/* The linearisation factor of GS_NEWTON_B (added): b = gamma*(1+w)*exp(w), in that evaluation order, at every
 * element of planes -1 .. nz+2 of a field laid out by gs_field_layout (interior, boundary and ghost planes, the
 * row padding included), so a Z-slab's B is current wherever its w is. w and b must not overlap. */
int gs_newton_bfac(const gs_level* L, double gamma, const double* w, double* b, hipStream_t stream);

/* dst[i] = value for i < n (Vector3::fill, src/cpu/Vector3.cpp:29-32). */
int gs_fill(double* dst, double value, int64_t n, hipStream_t stream);

/* dst[i] = src[i] for i < n (Vector3 copy-assignment: NewtonSolver.cpp:12 newtonF = f), non-temporal
 * streams; the buffers must not overlap unless dst == src. */
int gs_copy(double* dst, const double* src, int64_t n, hipStream_t stream);

/* y[i] += a*x[i] for i < n (a = +-1 is exact: the reference's Vector3 += / -=). */
int gs_axpy(double* y, const double* x, double a, int64_t n, hipStream_t stream);

/* The coarse end of the V-cycle in ONE launch of one workgroup (its levels stay in L2): lv[0..n)
 * are consecutive levels of the hierarchy, lv[0] the finest of them, whose f (and, NONLINEAR,
 * rest_v and v) the caller has already set. Runs CpuSolver::vcycle's recursion below that point
 * (src/cpu/CpuSolver.cpp:92-135: pre-smoothing, residual, full weighting, [FAS restV = v = R v,
 * f += A(restV)], the coarsest level's pre+post sweeps, then prolongation + correction and
 * post-smoothing back up to lv[0]) with the per-point expressions of the launchers above, so every
 * field is bit-identical to launching them one by one. Jacobi ping-pongs between v and v_alt: on
 * return every level's iterate is in v if pre+post is even, else in v_alt. v_zero: the level's
 * iterate is the zero iterate and v is not read. n <= gs_coarse_cycle_max_levels(); levels
 * unpartitioned (z0 = 0), each exactly half the previous one per axis (integer division); r is
 * needed on all but the last level, rest_v (NONLINEAR) on all but the first, newton_v (NEWTON) on
 * all. */
typedef struct {
    double *v, *v_alt, *f;
    double* r;        /* residual scratch */
    double* rest_v;   /* NONLINEAR: restricted iterate; else NULL */
    double* newton_v; /* NEWTON: the linearisation point (GS_NEWTON_B: its factor B); else NULL */
    gs_level geom;
    int v_zero;
} gs_coarse_level;
int gs_coarse_cycle_max_levels(void);
int gs_coarse_cycle(const gs_stencil* S, const gs_coarse_level* lv, int n, int mode, double omega, double gamma,
                    int pre, int post, hipStream_t stream);

const char* gs_strerror(int code);

/* (tuning variants, bandwidth probes and the rejected k_prr: include/gpusolve_diag.h) */
/* Library build tag (kernel variant names), for logs. */
const char* gs_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* GPUSOLVE_HIP_H */
