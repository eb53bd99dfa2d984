/* gpusolve_driver.h — C ABI of the GpuSolve-hip host driver (libgpusolve_driver.so).
 *
 * The reference's backend contract is a C++ one (a grid object + static solver functions selected
 * at compile time, src/main.cpp:5-13,88-111). This header exposes the same objects through a
 * plain C ABI (opaque handle, plain pointers and sizes) so non-C++ hosts (ctypes tests, bench.py,
 * a cgo/JNI wrapper) can drive the identical code path the GpuSolve-hip executable runs:
 *
 *   gs_grid_create         CpuGridData(const GridParams&)   src/cpu/CpuGridData.cpp:15-79
 *   gs_grid_solve          main's dispatch: NewtonSolver::solve (mode 2) else CpuSolver::solve
 *                                                          src/main.cpp:88-94
 *   gs_grid_vcycle         CpuSolver::vcycle                src/cpu/CpuSolver.cpp:85-139
 *   gs_grid_jacobi         CpuSolver::jacobi                src/cpu/CpuSolver.cpp:141-180
 *   gs_grid_residual_norm  CpuSolver::compResidual          src/cpu/CpuSolver.cpp:45-83
 *
 * Errors: functions return 0 / a non-NULL handle on success; otherwise gs_last_error() holds the
 * message the GpuSolve-hip executable would print after "Exception: ".
 */
#ifndef GPUSOLVE_DRIVER_H
#define GPUSOLVE_DRIVER_H

#include <stdint.h>
#include "gpusolve_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* GridParams (src/gridParams.h:29-47) in plain C. */
typedef struct {
    int64_t maxiter;
    double tol;
    int64_t dims[3];
    int mode; /* GS_LINEAR / GS_NONLINEAR / GS_NEWTON */
    int64_t pre, post;
    double omega, gamma;
    gs_stencil stencil;
} gs_params;

/* Parses the reference's 14-line config text. Returns 0, 1 (invalid mode), 2 (bad stencil). */
int gs_parse_config(const char* text, gs_params* out);

void* gs_grid_create(const gs_params* p); /* device-resident hierarchy on the current HIP device */
void gs_grid_destroy(void* grid);

/* Runs the solve selected by the mode. print: 0 silent, 1 reference stdout lines.
 * Writes up to cap residual values (initial, then one per V-cycle / Newton iteration) into hist
 * and their total count into *count. */
int gs_grid_solve(void* grid, int print, double* hist, int cap, int* count);

int gs_grid_vcycle(void* grid, double* residual);
int gs_grid_jacobi(void* grid, int level, int sweeps);
int gs_grid_residual_norm(void* grid, int level, double* norm);
int gs_grid_num_levels(void* grid);
/* 1 if the level's smoothing runs as fused sweep pairs (gs_jacobi_sweep2), else 0. */
int gs_grid_level_fused(void* grid, int level);
int gs_grid_level(void* grid, int level, gs_level* out);
/* field: 0 v (current iterate), 1 restV, 2 newtonV, 3 f, 4 r, 5 newtonF (level 0). NULL if absent. */
double* gs_grid_field(void* grid, int level, int field);
hipStream_t gs_grid_stream(void* grid);
/* Synchronous copies of a whole padded field to / from a dense host array laid out
 * [nz+2][ny+2][nx+2] (x fastest). */
int gs_grid_download(void* grid, int level, int field, double* host);
int gs_grid_upload(void* grid, int level, int field, const double* host);
int gs_grid_sync(void* grid);
/* Host cost of the ghost exchanges issued so far (Z-slab grids): total wall milliseconds spent inside
 * the exchange calls (RCCL: group start/end and the settle poll of the non-blocking communicator) and
 * the number of calls. Zero for single-GPU grids. */
int gs_grid_comm_stats(void* grid, double* halo_host_ms, int64_t* halo_calls);
/* The largest host cost of ONE exchange so far (issue + polls + settle; the pipelined sweep sequence
 * settles an exchange only before the next boundary planes, after the next interior is enqueued). */
int gs_grid_comm_stats_max(void* grid, double* halo_host_max_ms);
/* With GS_METRICS=1 in the environment when the grid was created: the "[gs] mlups=... gbps=...
 * pct_peak=... vcycle_ms=... cycles=... level_ms=..." line GpuSolve-hip prints after its solve (over
 * the V-cycles run so far), and the device ms per level and V-cycle. Non-zero if metrics are off. */
int gs_grid_metrics(void* grid, char* line, int cap, double* level_ms, int levels_cap);
/* Vector3::dump (src/cpu/Vector3.cpp:56-78) of a padded field: header "Px Py Pz" then "x y z value"
 * per point, x outermost, z innermost, values in the iostream default format (%g). path NULL or
 * empty (or not openable): the lines go to stdout without the header, as in the reference.
 * gs_dump_write formats a dense host array [pz][py][px] (x fastest); gs_grid_dump downloads first. */
int gs_dump_write(const double* host, int64_t px, int64_t py, int64_t pz, const char* path);
int gs_grid_dump(void* grid, int level, int field, const char* path);

/* Times `sweeps` level-`level` Jacobi sweeps with hipEvents on the grid's stream (after `warmup`
 * untimed sweeps); *ms = elapsed milliseconds of the timed sweeps. */
int gs_grid_time_jacobi(void* grid, int level, int warmup, int sweeps, float* ms);
/* Times `cycles` V-cycles (each including its norm readback) with a host clock; *ms total. */
int gs_grid_time_vcycles(void* grid, int cycles, double* ms, double* last_residual);

/* ---- Z-slab multi-GPU (new) ----
 * Ownership plan of every level for `nranks` ranks (pure host logic): distributed[l] = 1 when
 * level l is Z-slab partitioned; lo/hi[l*nranks + r] = rank r's owned global interior planes
 * (1-based, inclusive). min_points < 0 selects the default agglomeration threshold. Returns the
 * level count (at most max_levels entries are written). */
int gs_zslab_plan(const int64_t dims[3], int nranks, int64_t min_points, int max_levels, int* distributed,
                  int64_t* lo, int64_t* hi);
/* The Z-slab schedule of rank `rank` of `nranks` for the solve of p (construction, initial norm,
 * p->maxiter V-cycles / Newton iterations), produced by the driver's own V-cycle code in its trace mode
 * (no device touched): one line per kernel launch, ghost exchange, gather, norm reduction, swap and
 * zeroing, "op field=.. key=value ..." (ops: rhs pair sweep pro swap zero halo gather norm residual
 * resrestrict restrict prolongadd applyadd coarse copy newtonF axpy; L = level, z1..z2 = local planes,
 * c1..c2 = global coarse planes). Writes at most cap-1 bytes + NUL; *len = the full length. */
int gs_zslab_schedule(const gs_params* p, int nranks, int rank, int64_t min_points, char* buf, int64_t cap,
                      int64_t* len);
/* 128-byte RCCL unique id (rank 0 creates it, every rank passes the same bytes). */
int gs_rccl_unique_id(unsigned char uid[128]);
/* Grid whose levels are Z-slab partitioned over an RCCL communicator (one GPU per rank; the
 * current HIP device). The other gs_grid_* calls then run the distributed solver; fields and
 * levels describe this rank's slab; rank 0 prints. */
void* gs_grid_create_rccl(const gs_params* p, int rank, int nranks, const unsigned char uid[128]);
/* The same with an explicit RCCL CTA budget for this grid's communicator (ncclConfig_t::minCTAs = maxCTAs =
 * ctas: the workgroups RCCL's send/recv kernels take beside the interior sweep; 0: RCCL's own choice; -1: the
 * process default, GS_RCCL_CTAS or 64). gs_grid_create_rccl is ctas = -1. */
void* gs_grid_create_rccl_ctas(const gs_params* p, int rank, int nranks, const unsigned char uid[128], int ctas);
/* The CTA budget of the grid's RCCL communicator; -1 for single-GPU / loopback grids. */
int gs_grid_comm_ctas(void* grid);
/* NCCL_NCHANNELS_PER_PEER that gives one grouped ghost exchange (four send/recv per rank) the whole CTA budget
 * `ctas` (-1: the process default): ctas / 4, 0 for RCCL's default. RCCL reads the variable once per process,
 * so the LAUNCHER sets it (unless already set) before its first communicator — GpuSolve-hip's main and bench.py
 * do; the library never writes the process environment. */
int gs_rccl_channels_per_peer_hint(int ctas);
/* The id's file hand-off of a multi-process GpuSolve-hip run (one launcher, one node): rank 0
 * publishes (temporary file renamed into place), the others wait up to timeout_s for all 128 bytes.
 * 0 on success, else non-zero with gs_last_error(). */
int gs_uid_publish(const char* path, const unsigned char uid[128]);
int gs_uid_await(const char* path, double timeout_s, unsigned char uid[128]);
/* The id file GpuSolve-hip uses when GS_UID_FILE is unset: /tmp/gpusolve-uid-<parent pid>-<MASTER_PORT>,
 * plus -<TORCHELASTIC_RUN_ID>-a<TORCHELASTIC_RESTART_COUNT> under torchrun, so that each restart attempt
 * has its own file. Writes at most cap-1 bytes + NUL; returns the full length. */
int gs_uid_default_path(char* buf, int cap);
/* Single-process emulation of an nranks Z-slab run on the current device: nranks threads, each a
 * rank with its own slab and streams, device-to-device copies as the exchange. Runs `sweeps`
 * level-0 Jacobi sweeps, then (solve != 0) the solve of p. Writes rank 0's residual history and
 * the assembled level-0 v (dense [nz+2][ny+2][nx+2], interior planes only; NULL to skip).
 * min_points as in gs_zslab_plan. For testing the distributed path on one GPU. */
int gs_zslab_loopback_run(const gs_params* p, int nranks, int64_t min_points, int sweeps, int solve, double* hist,
                          int cap, int* count, double* v_host);

/* ---- failure-detection self-tests (host logic only; no GPU) ----
 * gs_debug_bounded_wait: the bounded wait that settles every RCCL call and sync (gs_comm.hpp),
 * driven by a fake poll: scenario 0 completes at poll k, 1 reports ncclInternalError at poll k,
 * 2 never completes (times out after timeout_s). Returns 0 on completion, 1 with the message in msg.
 * gs_debug_loopback_abort: nranks threads meet at loopback-hub barriers and failing_rank throws;
 * returns how many threads unwound (nranks = none left hanging); gs_last_error() = the first error. */
int gs_debug_bounded_wait(int scenario, int k, double timeout_s, char* msg, int cap);
int gs_debug_loopback_abort(int nranks, int failing_rank);

const char* gs_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* GPUSOLVE_DRIVER_H */
