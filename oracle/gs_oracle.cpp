// gs_oracle.cpp — CPU ORACLE, TEST INFRASTRUCTURE ONLY.
//
// A from-scratch restatement of the reference CPU solver's numerics (Bricktricker/gpu-solve
// src/cpu, snapshot 2025-02-27). Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load this library; the product path (libgpusolve_hip / GpuSolve-hip)
// never links or calls it.
//
// Pinned against the reference itself: tests/golden/* were produced by oracle/_ref/ref_probe,
// which links the reference's own src/cpu/*.cpp (see tests/golden/make_golden.py), and
// tests/test_oracle_golden.py checks this restatement against every one of them.
//
// Storage follows the reference's Vector3 (src/cpu/Vector3.cpp:16,24): padded (nx+2, ny+2, nz+2)
// doubles, z unit-stride: idx = z + y*Pz + x*Pz*Py.
//
// Every arithmetic expression below is evaluated in the same order as the reference so that
// g++ (no FMA contraction on x86-64 without -march) reproduces it bit for bit; only the order of
// the OpenMP sum-of-squares reductions differs (≈1e-14 relative).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#include <omp.h>

extern "C" {

typedef struct {
    double s[7];
    int ox[7], oy[7], oz[7];
} gso_stencil;

} // extern "C"

namespace {

struct Dims {
    int64_t nx, ny, nz; // interior extents
    int64_t Px() const { return nx + 2; }
    int64_t Py() const { return ny + 2; }
    int64_t Pz() const { return nz + 2; }
    int64_t size() const { return Px() * Py() * Pz(); }
    // reference layout, src/cpu/Vector3.cpp:16
    int64_t at(int64_t x, int64_t y, int64_t z) const { return z + Pz() * (y + Py() * x); }
};

// src/cpu/CpuGridData.cpp:7-12 (left-to-right evaluation kept)
inline double rhs_f0(double x) { return 100 * x * (x - 1.0) * x * (x - 1.0) * x * (x - 1.0) * x * (x - 1.0); }
inline double rhs_f2(double x) { return 100.0 * 4.0 * (x - 1.0) * (x - 1.0) * x * x * (14.0 * x * x - 14.0 * x + 3); }

inline double stencil_apply(const gso_stencil& S, const Dims& d, const double* u, int64_t x, int64_t y, int64_t z)
{
    double acc = 0.0;
    for (int i = 0; i < 7; i++) acc += S.s[i] * u[d.at(x + S.ox[i], y + S.oy[i], z + S.oz[i])];
    return acc;
}

enum { LINEAR = 0, NONLINEAR = 1, NEWTON = 2 };

// Residual r = f - A(v) on the interior, returns sqrt(sum r^2).  src/cpu/CpuSolver.cpp:45-83
double residual(const gso_stencil& S, const Dims& d, double h, int mode, double gamma, const double* v,
                const double* f, const double* w, double* r)
{
    double sumsq = 0.0;
#pragma omp parallel for schedule(static, 8) reduction(+ : sumsq)
    for (int64_t x = 1; x <= d.nx; x++)
        for (int64_t y = 1; y <= d.ny; y++)
            for (int64_t z = 1; z <= d.nz; z++) {
                const int64_t p = d.at(x, y, z);
                double s = stencil_apply(S, d, v, x, y, z);
                s /= h * h;
                if (mode == NEWTON) {
                    const double ew = std::exp(w[p]);
                    s += gamma * (1 + w[p]) * v[p] * ew;
                } else if (mode == NONLINEAR) {
                    const double ev = std::exp(v[p]);
                    const double nl = gamma * v[p] * ev;
                    s += nl;
                }
                const double rr = f[p] - s;
                if (r) r[p] = rr;
                sumsq += rr * rr;
            }
    return std::sqrt(sumsq);
}

// k damped-Jacobi sweeps, each = residual of the old iterate then a pointwise update.
// src/cpu/CpuSolver.cpp:141-180.  r is scratch (the reference writes level.r).
void jacobi(const gso_stencil& S, const Dims& d, double h, int mode, double omega, double gamma, int sweeps,
            double* v, const double* f, const double* w, double* r)
{
    const double h2 = h * h;
    const double preFac = S.s[0] / h2;
    const double alpha = h2 / S.s[0];
    for (int it = 0; it < sweeps; it++) {
        residual(S, d, h, mode, gamma, v, f, w, r);
#pragma omp parallel for schedule(static, 8)
        for (int64_t x = 1; x <= d.nx; x++)
            for (int64_t y = 1; y <= d.ny; y++)
                for (int64_t z = 1; z <= d.nz; z++) {
                    const int64_t p = d.at(x, y, z);
                    double nv;
                    if (mode == LINEAR) {
                        nv = v[p] + omega * (alpha * r[p]);
                    } else {
                        const double u = (mode == NONLINEAR) ? v[p] : w[p];
                        const double eu = std::exp(u);
                        const double den = preFac + gamma * (1 + u) * eu;
                        nv = v[p] + omega * (r[p] / den);
                    }
                    v[p] = nv;
                }
    }
}

// FAS coarse operator out = A(u)/h^2 + gamma*u*exp(u) on the interior.  src/cpu/CpuSolver.cpp:182-208
void apply_op(const gso_stencil& S, const Dims& d, double h, double gamma, const double* u, double* out)
{
#pragma omp parallel for schedule(static, 8)
    for (int64_t x = 1; x <= d.nx; x++)
        for (int64_t y = 1; y <= d.ny; y++)
            for (int64_t z = 1; z <= d.nz; z++) {
                const int64_t p = d.at(x, y, z);
                double s = stencil_apply(S, d, u, x, y, z);
                s /= h * h;
                const double nl = gamma * u[p] * std::exp(u[p]);
                s += nl;
                out[p] = s;
            }
}

// 27-point full weighting onto the coarse interior.  src/cpu/CpuSolver.cpp:211-238
void restrict_fw(const double* fine, const Dims& fd, double* coarse, const Dims& cd)
{
#pragma omp parallel for schedule(static, 8)
    for (int64_t x = 1; x <= cd.nx; x++)
        for (int64_t y = 1; y <= cd.ny; y++)
            for (int64_t z = 1; z <= cd.nz; z++) {
                double acc = 0.0;
                for (int a = -1; a <= 1; a++)
                    for (int b = -1; b <= 1; b++)
                        for (int c = -1; c <= 1; c++) {
                            const double wgt = 0.125 * ((2.0 - std::abs(a)) / 2.0) * ((2.0 - std::abs(b)) / 2.0) *
                                               ((2.0 - std::abs(c)) / 2.0);
                            acc += wgt * fine[fd.at(2 * x + a, 2 * y + b, 2 * z + c)];
                        }
                coarse[cd.at(x, y, z)] = acc;
            }
}

// Trilinear prolongation coarse v -> fine e: injection, then x, y, z linear passes in that order.
// src/cpu/CpuSolver.cpp:240-290.  Index P-1 on each axis is never written.
void interpolate(const double* coarse, const Dims& cd, double* e, const Dims& fd)
{
    const int64_t Px = fd.Px(), Py = fd.Py(), Pz = fd.Pz();
#pragma omp parallel for schedule(static, 4)
    for (int64_t x = 0; x < Px - 1; x += 2)
        for (int64_t y = 0; y < Py - 1; y += 2)
            for (int64_t z = 0; z < Pz - 1; z += 2) e[fd.at(x, y, z)] = coarse[cd.at(x / 2, y / 2, z / 2)];
#pragma omp parallel for schedule(static, 4)
    for (int64_t x = 0; x < Px - 2; x += 2)
        for (int64_t y = 0; y < Py; y += 2)
            for (int64_t z = 0; z < Pz; z += 2)
                e[fd.at(x + 1, y, z)] = 0.5 * e[fd.at(x, y, z)] + 0.5 * e[fd.at(x + 2, y, z)];
#pragma omp parallel for schedule(static, 4)
    for (int64_t x = 0; x < Px; x++)
        for (int64_t y = 0; y + 2 < Py; y += 2)
            for (int64_t z = 0; z < Pz; z += 2)
                e[fd.at(x, y + 1, z)] = 0.5 * e[fd.at(x, y, z)] + 0.5 * e[fd.at(x, y + 2, z)];
#pragma omp parallel for schedule(static, 4)
    for (int64_t x = 0; x < Px; x++)
        for (int64_t y = 0; y < Py; y++)
            for (int64_t z = 0; z + 2 < Pz; z += 2)
                e[fd.at(x, y, z + 1)] = 0.5 * e[fd.at(x, y, z)] + 0.5 * e[fd.at(x, y, z + 2)];
}

// Newton outer residual f0 = newtonF - N(newtonV); returns its norm.  src/cpu/NewtonSolver.cpp:48-81
double newton_F(const gso_stencil& S, const Dims& d, double h, double gamma, const double* w, const double* F,
                double* f)
{
    double sumsq = 0.0;
#pragma omp parallel for schedule(static, 8) reduction(+ : sumsq)
    for (int64_t x = 1; x <= d.nx; x++)
        for (int64_t y = 1; y <= d.ny; y++)
            for (int64_t z = 1; z <= d.nz; z++) {
                const int64_t p = d.at(x, y, z);
                double s = stencil_apply(S, d, w, x, y, z);
                s /= h * h;
                const double ew = std::exp(w[p]);
                const double nl = gamma * w[p] * ew;
                s += nl;
                const double val = F[p] - s;
                f[p] = val;
                sumsq += val * val;
            }
    return std::sqrt(sumsq);
}

// Level-0 right-hand side.  src/cpu/CpuGridData.cpp:44-78
void init_rhs(const Dims& d, double h, int mode, double gamma, double* f)
{
    if (mode == LINEAR) {
        // interior point (i+1, j+1, k+1) evaluated at (i*h, j*h, k*h): the reference's offset is kept
        for (int64_t i = 0; i < d.nx; i++)
            for (int64_t j = 0; j < d.ny; j++)
                for (int64_t k = 0; k < d.nz; k++) {
                    const double x = (int)i * h, y = (int)j * h, z = (int)k * h;
                    f[d.at(i + 1, j + 1, k + 1)] =
                        -(rhs_f2(x) * rhs_f0(y) * rhs_f0(z) + rhs_f0(x) * rhs_f2(y) * rhs_f0(z) +
                          rhs_f0(x) * rhs_f0(y) * rhs_f2(z));
                }
    } else {
        for (int64_t i = 0; i < d.Px(); i++)
            for (int64_t j = 0; j < d.Py(); j++)
                for (int64_t k = 0; k < d.Pz(); k++) {
                    const double x = (int)i * h, y = (int)j * h, z = (int)k * h;
                    const double ux = x - x * x, uy = y - y * y, uz = z - z * z;
                    f[d.at(i, j, k)] = 2.0 * ((y - y * y) * (z - z * z) + (x - x * x) * (z - z * z) +
                                              (x - x * x) * (y - y * y)) +
                                       gamma * ux * uy * uz * std::exp(ux * uy * uz);
                }
    }
}

void add_into(double* a, const double* b, int64_t n, double sign)
{
    if (sign > 0) {
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; i++) a[i] += b[i];
    } else {
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; i++) a[i] -= b[i];
    }
}

// ---------------------------------------------------------------------------------------------
// The level hierarchy and drivers (src/cpu/CpuGridData.cpp:15-42, CpuSolver.cpp:12-43/85-139,
// NewtonSolver.cpp:10-108).
struct Level {
    Dims d;
    double h;
    std::vector<double> v, restV, newtonV, f, r, e;
};

struct Grid {
    gso_stencil S;
    int mode;
    int64_t maxiter;
    double tol, omega, gamma;
    int64_t pre, post;
    std::vector<Level> L;
    std::vector<double> newtonF;
    int print;                     // 0 quiet, 1 print reference-format lines
    std::vector<double> history;   // [initial, after cycle 0, ...] of the outermost solve
};

Grid* make_grid(const gso_stencil* S, const int64_t dims[3], int mode, int64_t maxiter, double tol, double omega,
                double gamma, int64_t pre, int64_t post)
{
    Grid* g = new Grid;
    g->S = *S;
    g->mode = mode;
    g->maxiter = maxiter;
    g->tol = tol;
    g->omega = omega;
    g->gamma = gamma;
    g->pre = pre;
    g->post = post;
    g->print = 0;
    const int64_t mn = std::min(std::min(dims[0], dims[1]), dims[2]);
    const int nlev = (int)std::floor(std::log((double)mn) / std::log(2.0)) + 1;
    g->L.resize(nlev);
    Dims d{dims[0], dims[1], dims[2]};
    for (int l = 0; l < nlev; l++) {
        if (l > 0) d = Dims{d.nx / 2, d.ny / 2, d.nz / 2};
        Level& lv = g->L[l];
        lv.d = d;
        lv.h = 1.0 / (d.ny + 1);
        const int64_t n = d.size();
        lv.v.assign(n, 0.0);
        lv.restV.assign(n, 0.0);
        lv.newtonV.assign(n, 0.0);
        lv.f.assign(n, 0.0);
        lv.r.assign(n, 0.0);
        if (l + 1 != nlev) lv.e.assign(n, 0.0);
    }
    // main.cpp:84 uses h = 1/(Y+1) for the RHS, identical to level 0's h
    init_rhs(g->L[0].d, 1.0 / (dims[1] + 1), mode, gamma, g->L[0].f.data());
    return g;
}

double g_residual(Grid& g, int l)
{
    Level& lv = g.L[l];
    return residual(g.S, lv.d, lv.h, g.mode, g.gamma, lv.v.data(), lv.f.data(), lv.newtonV.data(), lv.r.data());
}

void g_jacobi(Grid& g, int l, int64_t sweeps)
{
    Level& lv = g.L[l];
    jacobi(g.S, lv.d, lv.h, g.mode, g.omega, g.gamma, (int)sweeps, lv.v.data(), lv.f.data(), lv.newtonV.data(),
           lv.r.data());
}

double vcycle(Grid& g)
{
    const int nl = (int)g.L.size();
    for (int l = 0; l + 1 < nl; l++) {
        g_jacobi(g, l, g.pre);
        Level& fine = g.L[l];
        Level& crs = g.L[l + 1];
        g_residual(g, l);
        restrict_fw(fine.r.data(), fine.d, crs.f.data(), crs.d);
        if (g.mode != NONLINEAR) {
            std::fill(crs.v.begin(), crs.v.end(), 0.0);
        } else {
            restrict_fw(fine.v.data(), fine.d, crs.restV.data(), crs.d);
            restrict_fw(fine.v.data(), fine.d, crs.v.data(), crs.d);
            apply_op(g.S, crs.d, crs.h, g.gamma, crs.restV.data(), crs.r.data());
            add_into(crs.f.data(), crs.r.data(), crs.d.size(), +1);
        }
    }
    g_jacobi(g, nl - 1, g.pre + g.post);
    for (int l = nl - 1; l > 0; l--) {
        Level& crs = g.L[l];
        Level& fine = g.L[l - 1];
        if (g.mode == NONLINEAR) add_into(crs.v.data(), crs.restV.data(), crs.d.size(), -1);
        interpolate(crs.v.data(), crs.d, fine.e.data(), fine.d);
        add_into(fine.v.data(), fine.e.data(), fine.d.size(), +1);
        g_jacobi(g, l - 1, g.post);
    }
    return g_residual(g, 0);
}

double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void solve(Grid& g, int print, std::vector<double>* hist)
{
    const double r0 = g_residual(g, 0);
    if (hist) hist->push_back(r0);
    if (print) std::printf(print == 2 ? "Inital residual: %.17g\n" : "Inital residual: %g\n", r0);
    for (int64_t i = 0; i < g.maxiter; i++) {
        const double t0 = now_ms();
        const double res = vcycle(g);
        if (hist) hist->push_back(res);
        if (print)
            std::printf(print == 2 ? "iter: %lld residual: %.17g Took %lldms\n" : "iter: %lld residual: %g Took %lldms\n",
                        (long long)i, res, (long long)(now_ms() - t0));
        if (res <= r0 / (1.0 / g.tol)) return;
    }
}

double newton_compF(Grid& g)
{
    Level& l0 = g.L[0];
    return newton_F(g.S, l0.d, l0.h, g.gamma, l0.newtonV.data(), g.newtonF.data(), l0.f.data());
}

void newton_solve(Grid& g, int print, std::vector<double>* hist)
{
    g.newtonF = g.L[0].f;
    const double r0 = newton_compF(g);
    if (hist) hist->push_back(r0);
    if (print) std::printf(print == 2 ? "Inital newton residual: %.17g\n" : "Inital newton residual: %g\n", r0);
    for (int64_t i = 0; i < g.maxiter; i++) {
        const double t0 = now_ms();
        newton_compF(g);
        std::fill(g.L[0].v.begin(), g.L[0].v.end(), 0.0);
        // findError: restrict newtonV to levels 1..L-2 (the coarsest keeps its newtonV), inner solve
        const int nl = (int)g.L.size();
        for (int l = 1; l + 1 < nl; l++)
            restrict_fw(g.L[l - 1].newtonV.data(), g.L[l - 1].d, g.L[l].newtonV.data(), g.L[l].d);
        const int64_t mi = g.maxiter;
        const double tl = g.tol;
        g.maxiter = 10;
        g.tol = 0.1;
        solve(g, 0, nullptr);
        g.maxiter = mi;
        g.tol = tl;
        add_into(g.L[0].newtonV.data(), g.L[0].v.data(), g.L[0].d.size(), +1);
        const double res = newton_compF(g);
        if (hist) hist->push_back(res);
        if (print)
            std::printf(print == 2 ? "newton iter: %lld residual: %.17g Took %lldms\n"
                                   : "newton iter: %lld residual: %g Took %lldms\n",
                        (long long)i, res, (long long)(now_ms() - t0));
        if (res <= r0 / (1.0 / tl)) return;
    }
}

} // namespace

// ---------------------------------------------------------------------------------------------
// C ABI for tests/ (ctypes) and for the oracle CLI.  Arrays are caller-owned, reference layout.
extern "C" {

int gso_num_threads(void) { return omp_get_max_threads(); }

double gso_residual(const gso_stencil* S, const int64_t n[3], double h, int mode, double gamma, const double* v,
                    const double* f, const double* w, double* r)
{
    return residual(*S, Dims{n[0], n[1], n[2]}, h, mode, gamma, v, f, w, r);
}

void gso_jacobi(const gso_stencil* S, const int64_t n[3], double h, int mode, double omega, double gamma, int sweeps,
                double* v, const double* f, const double* w, double* r_scratch)
{
    jacobi(*S, Dims{n[0], n[1], n[2]}, h, mode, omega, gamma, sweeps, v, f, w, r_scratch);
}

void gso_apply_op(const gso_stencil* S, const int64_t n[3], double h, double gamma, const double* u, double* out)
{
    apply_op(*S, Dims{n[0], n[1], n[2]}, h, gamma, u, out);
}

void gso_restrict(const double* fine, const int64_t fn[3], double* coarse, const int64_t cn[3])
{
    restrict_fw(fine, Dims{fn[0], fn[1], fn[2]}, coarse, Dims{cn[0], cn[1], cn[2]});
}

void gso_interpolate(const double* coarse, const int64_t cn[3], double* e, const int64_t fn[3])
{
    interpolate(coarse, Dims{cn[0], cn[1], cn[2]}, e, Dims{fn[0], fn[1], fn[2]});
}

double gso_newton_F(const gso_stencil* S, const int64_t n[3], double h, double gamma, const double* w, const double* F,
                    double* f)
{
    return newton_F(*S, Dims{n[0], n[1], n[2]}, h, gamma, w, F, f);
}

void gso_rhs(const int64_t n[3], double h, int mode, double gamma, double* f)
{
    init_rhs(Dims{n[0], n[1], n[2]}, h, mode, gamma, f);
}

void* gso_grid_create(const gso_stencil* S, const int64_t dims[3], int mode, int64_t maxiter, double tol, double omega,
                      double gamma, int64_t pre, int64_t post)
{
    return make_grid(S, dims, mode, maxiter, tol, omega, gamma, pre, post);
}

void gso_grid_destroy(void* g) { delete static_cast<Grid*>(g); }

int gso_grid_levels(void* gp) { return (int)static_cast<Grid*>(gp)->L.size(); }

void gso_grid_level_info(void* gp, int l, int64_t dims_out[3], double* h_out)
{
    Level& lv = static_cast<Grid*>(gp)->L[l];
    dims_out[0] = lv.d.nx;
    dims_out[1] = lv.d.ny;
    dims_out[2] = lv.d.nz;
    *h_out = lv.h;
}

// field: 0 v, 1 restV, 2 newtonV, 3 f, 4 r, 5 e
double* gso_grid_field(void* gp, int l, int field)
{
    Level& lv = static_cast<Grid*>(gp)->L[l];
    std::vector<double>* fs[6] = {&lv.v, &lv.restV, &lv.newtonV, &lv.f, &lv.r, &lv.e};
    return fs[field]->empty() ? nullptr : fs[field]->data();
}

double gso_grid_vcycle(void* gp) { return vcycle(*static_cast<Grid*>(gp)); }

// Runs the solve for the grid's mode; writes up to cap history entries, returns the count.
int gso_grid_solve(void* gp, int print, double* hist, int cap)
{
    Grid& g = *static_cast<Grid*>(gp);
    std::vector<double> h;
    if (g.mode == NEWTON) newton_solve(g, print, &h);
    else solve(g, print, &h);
    const int n = std::min<int>((int)h.size(), cap);
    if (hist) std::memcpy(hist, h.data(), sizeof(double) * n);
    return (int)h.size();
}

} // extern "C"

// ---------------------------------------------------------------------------------------------
// Timing helpers for bench.py's cpu_baseline leg (kind "port"): level-0 Jacobi sweeps and V-cycles.
extern "C" {

// Returns seconds for `sweeps` Jacobi sweeps on level 0 of an (X,Y,Z) grid (one warm-up sweep first).
double gso_time_jacobi(const gso_stencil* S, const int64_t dims[3], int mode, int sweeps)
{
    Grid* g = make_grid(S, dims, mode, 1, 0.0, 0.8, 1.0, 2, 2);
    g_jacobi(*g, 0, 1);
    const double t0 = now_ms();
    g_jacobi(*g, 0, sweeps);
    const double t1 = now_ms();
    delete g;
    return (t1 - t0) * 1e-3;
}

// Returns seconds per V-cycle (2+2) averaged over `cycles` after one warm-up cycle.
double gso_time_vcycle(const gso_stencil* S, const int64_t dims[3], int mode, int cycles, double* last_res)
{
    Grid* g = make_grid(S, dims, mode, 1, 0.0, 0.8, 1.0, 2, 2);
    vcycle(*g);
    const double t0 = now_ms();
    double r = 0;
    for (int c = 0; c < cycles; c++) r = vcycle(*g);
    const double t1 = now_ms();
    if (last_res) *last_res = r;
    delete g;
    return (t1 - t0) * 1e-3 / cycles;
}

} // extern "C"
