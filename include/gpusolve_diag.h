/* gpusolve_diag.h — C ABI of libgpusolve_diag.so: measurement and tuning code that is NOT part of the
 * product (include/gpusolve_hip.h). Loaded only by tools/, tests/ and bench.py's measured-ceiling leg.
 * Conventions (layout, stencil, streams, errors) as in gpusolve_hip.h.
 */
#ifndef GPUSOLVE_DIAG_H
#define GPUSOLVE_DIAG_H

#include "gpusolve_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* k_prr (built, bit-identical, measured SLOWER than the two passes the driver runs: DESIGN.md §9).
 * The first pre-smoothing pair of a 2-sweep pre-smoothing, the residual of its result and the full
 * weighting in one pass: v_out = S(S(v_in)), coarse_a (and coarse_b if not NULL) = R(f - A(v_out)) on
 * the coarse interior, partials (may be NULL) = gs_jacobi_sweep2_restrict_num_partials per-block sums
 * of r^2 of f - A(v_in). Bit-identical to gs_jacobi_sweep2 followed by gs_residual_restrict (the norm
 * in this kernel's block order). Replaces CpuSolver.cpp:94-99 (jacobi(pre = 2), compResidual,
 * restrict). Supported (gs_jacobi_sweep2_restrict_supported != 0) for LINEAR levels with the unit
 * 7-point stencil (canonical order, neighbour weights -1, |s0| >= 1), rows <= 512 points, z0 = 0, and
 * coarse = fine / 2 per axis; GS_EINVAL otherwise. */
int gs_jacobi_sweep2_restrict_supported(const gs_stencil* S, const gs_level* fine, const gs_level* coarse, int mode);
int gs_jacobi_sweep2_restrict(const gs_stencil* S, const gs_level* fine, double omega, const double* v_in,
                              double* v_out, const double* f, double* partials, double* coarse_a, double* coarse_b,
                              const gs_level* coarse, hipStream_t stream);
int64_t gs_jacobi_sweep2_restrict_num_partials(const gs_stencil* S, const gs_level* fine, const gs_level* coarse);
/* Measured and not adopted (r04, DESIGN.md §9: 122 vs 125 us at a 256^3 level, 38 vs 28 us at 128^3):
 * a coarse level's first down-leg step from v = 0 (LINEAR, canonical unit stencil, whole levels of rows <=
 * 512 points, Coef-style finite weights and h^2 normal): the zero-iterate pair's first sweep is pointwise in
 * f there, so ONE pass reads f once and writes v_out = S(S(0)) and coarse_f = R(f - A v_out)
 *   == two jacobi sweeps from v = 0 + compResidual + restrict          CpuSolver.cpp:94-99,114-116,141-180,211-238
 * bit-identical to gs_jacobi_sweep2 (v_in NULL) + gs_residual_restrict. Only interior points of v_out are
 * written; coarse = fine / 2 per axis. */
int gs_smooth2_restrict_zero_supported(const gs_stencil* S, const gs_level* fine, const gs_level* coarse, int mode);
int gs_smooth2_restrict_zero(const gs_stencil* S, const gs_level* fine, double omega, double* v_out, const double* f,
                             double* coarse_f, const gs_level* coarse, hipStream_t stream);

/* ---- tuning / diagnostics (tools/kbench.py) ----
 * Alternative tilings of the LINEAR fused sweep (bit-identical results), and a streaming
 * out = a + 0.8*b kernel (24 B per element, the smoother's byte pattern) for the achievable
 * HBM ceiling. n must be even and the arrays 16-B aligned. */
int gs_debug_num_variants(void);
const char* gs_debug_variant_name(int variant);
int gs_debug_sweep_variant(int variant, const gs_stencil* S, const gs_level* L, double omega, const double* v_in,
                           double* v_out, const double* f, hipStream_t stream);
/* fast[i] = the kernels' a[i] / hh (3-operation path where it applies), ref[i] = plain division. */
int gs_debug_div_check(const double* a, int64_t n, double hh, double* fast, double* ref, hipStream_t stream);
/* q[i] = the GS_NEWTON_B kernels' Jacobi quotient r[i] / den[i] (nb_quot: den's one-step refined reciprocal). */
int gs_debug_nb_quot(const double* r, const double* den, int64_t n, double* q, hipStream_t stream);
/* Fused-pair shape variants (LINEAR, level boundaries on both z sides; zc = 0: default chunk). */
int gs_debug_num_pair_variants(void);
const char* gs_debug_pair_variant_name(int variant);
int gs_debug_pair_variant(int variant, const gs_stencil* S, const gs_level* L, double omega, const double* v_in,
                          double* v_out, const double* f, int zc, hipStream_t stream);
int gs_debug_stream_triad(double* out, const double* a, const double* b, int64_t n, hipStream_t stream);
/* Streaming ceilings: kind 0 read a, 1 write out, 2 copy, 3 triad; unroll 1 or 4 dwordx4 per thread,
 * nt = non-temporal, `blocks` workgroups of 256 threads (grid-stride); blocks <= 0 (kinds 0-3): a grid that
 * covers the array once, no grid-stride loop, unroll 1, 2 or 4 dwordx4 per thread. Kind 4: a non-temporal copy
 * at the resource footprint of RCCL's transport kernels (256 VGPRs, 37 KB of LDS per workgroup;
 * unroll / nt ignored), the stand-in exchange of tools/exchange_probe.py. Kind 5: one wave that sleeps n x
 * s_sleep(127) (~3.4 us each), touching no memory (out / a / b / blocks ignored). */
int gs_debug_bw(int kind, int unroll, int nt, int blocks, double* out, const double* a, const double* b, int64_t n,
                double* sink, hipStream_t stream);
/* The LINEAR pair's memory skeleton without its arithmetic (k_march): k_tb2y's tiles, z-march over chunks of zc
 * planes, loads (pfd = 1 or 2 plane steps in flight) and stores, outputs a pointwise mix of the loaded values;
 * bar: a workgroup barrier per plane step; nts / ntf: non-temporal stores / f loads (ntf 2: only the rows
 * stored are loaded, pfd 2, nt stores; ntf 3 / 4 / 5: every block at most 2 / 4 / 8 plane steps ahead of the
 * slowest (a relaxed agent-scope counter in out's plane -1, bounded spins; at most 256 blocks), pfd 2, nt stores;
 * ntf 6 / 7: 1 / 4 rows per wave (2- / 8-row tiles; pfd 2 / 1), barrier, nt stores). Levels of nx <= 512 points,
 * ny a multiple of 4. 24 B per point. */
/* One workgroup of `threads` (512 / 1024) running `phases` rounds of [work -> store -> barrier]; work 0: none, 1: a
 * 7-point LDS stencil and a dependent FP64 chain, 2: the same from global memory g (>= 8192 doubles) with a global
 * store. The per-phase floor of the one-launch coarse cycle. */
int gs_debug_phase_probe(int work, int threads, int phases, double* g, double* sink, hipStream_t stream);
int gs_debug_march(int pfd, int bar, int nts, int ntf, int zc, const gs_level* L, const double* v, const double* f,
                   double* out, hipStream_t stream);

/* The production LINEAR pair with per-block timestamps (4 doubles per block in ts: start and end wall
 * clock at 100 MHz, hardware block index, HW_ID); zc > 0 overrides the plan's z-chunk. */
int gs_debug_pair_timestamps(const gs_stencil* S, const gs_level* L, double omega, const double* v_in, double* v_out,
                             const double* f, int zc, double* ts, hipStream_t stream);
int64_t gs_debug_pair_blocks(const gs_stencil* S, const gs_level* L, int zc);

/* The LINEAR pair (k_tb2y, rows of <= 512 points, unit stencils) in another shape: ry output rows per y-wave (1, 2),
 * pfd plane steps of prefetch (1, 2), wpe waves per SIMD the register allocation allows (0: one, as the product; 3;
 * 4: two 8-wave blocks per CU), zc planes per chunk (even). Output bit-identical to gs_jacobi_sweep2's. */
int gs_debug_pair_shape(const gs_stencil* S, const gs_level* L, double omega, const double* v_in, double* v_out,
                        const double* f, int ry, int pfd, int wpe, int zc, hipStream_t stream);

/* Timing only: the production LINEAR pair with the planes marched in descending order (reverse != 0; the
 * z-terms enter the sum swapped, so the values are not the sweep's). */
int gs_debug_pair_reverse(const gs_stencil* S, const gs_level* L, double omega, const double* v_in, double* v_out,
                          const double* f, int reverse, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* GPUSOLVE_DIAG_H */
