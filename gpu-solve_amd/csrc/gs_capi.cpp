// gs_capi.cpp — extern "C" facade of the host driver (include/gpusolve_driver.h).
#include <chrono>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "gpusolve_driver.h"
#include "gs_grid.hpp"

namespace {

thread_local std::string g_err;

template <class F>
int guarded(F&& f)
{
    try {
        f();
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return 1;
    }
}

gs::GridParams toParams(const gs_params* p)
{
    gs::GridParams g;
    g.maxiter = (std::size_t)p->maxiter;
    g.tol = p->tol;
    g.gridDim = {(std::size_t)p->dims[0], (std::size_t)p->dims[1], (std::size_t)p->dims[2]};
    g.mode = static_cast<gs::GridParams::Mode>(p->mode);
    g.preSmoothing = (std::size_t)p->pre;
    g.postSmoothing = (std::size_t)p->post;
    g.omega = p->omega;
    g.gamma = p->gamma;
    for (int i = 0; i < 7; i++) {
        g.stencil.values[i] = p->stencil.s[i];
        g.stencil.offsets[i] = std::make_tuple(p->stencil.ox[i], p->stencil.oy[i], p->stencil.oz[i]);
    }
    g.h = 1.0 / (g.gridDim[1] + 1);
    return g;
}

gs::HipGridData& G(void* h) { return *static_cast<gs::HipGridData*>(h); }

} // namespace

extern "C" {

int gs_parse_config(const char* text, gs_params* out)
{
    gs::GridParams g;
    const gs::ConfigStatus st = gs::parseConfigText(text ? text : "", g);
    if (st == gs::ConfigStatus::InvalidMode) return 1;
    if (st == gs::ConfigStatus::BadStencil) return 2;
    out->maxiter = (int64_t)g.maxiter;
    out->tol = g.tol;
    for (int i = 0; i < 3; i++) out->dims[i] = (int64_t)g.gridDim[i];
    out->mode = (int)g.mode;
    out->pre = (int64_t)g.preSmoothing;
    out->post = (int64_t)g.postSmoothing;
    out->omega = g.omega;
    out->gamma = g.gamma;
    for (int i = 0; i < 7; i++) {
        out->stencil.s[i] = g.stencil.values[i];
        out->stencil.ox[i] = g.stencil.getXOffset(i);
        out->stencil.oy[i] = g.stencil.getYOffset(i);
        out->stencil.oz[i] = g.stencil.getZOffset(i);
    }
    return 0;
}

void* gs_grid_create(const gs_params* p)
{
    if (!p) {
        g_err = "null params";
        return nullptr;
    }
    try {
        return new gs::HipGridData(toParams(p));
    } catch (const std::exception& e) {
        g_err = e.what();
        return nullptr;
    }
}

void gs_grid_destroy(void* grid) { delete static_cast<gs::HipGridData*>(grid); }

int gs_grid_solve(void* grid, int print, double* hist, int cap, int* count)
{
    return guarded([&] {
        auto& g = G(grid);
        std::vector<double> h;
        g.printProgress = print != 0;
        if (g.mode == gs::GridParams::NEWTON) {
            gs::NewtonSolver::history = &h;
            try {
                if (print) gs::NewtonSolver::solve(g);
                else {
                    // NewtonSolver::solve prints unconditionally (reference behaviour); silence it here
                    std::streambuf* old = std::cout.rdbuf(nullptr);
                    try {
                        gs::NewtonSolver::solve(g);
                    } catch (...) {
                        std::cout.rdbuf(old);
                        throw;
                    }
                    std::cout.rdbuf(old);
                }
            } catch (...) {
                gs::NewtonSolver::history = nullptr;
                throw;
            }
            gs::NewtonSolver::history = nullptr;
        } else {
            gs::HipSolver::history = &h;
            try {
                gs::HipSolver::solve(g);
            } catch (...) {
                gs::HipSolver::history = nullptr;
                throw;
            }
            gs::HipSolver::history = nullptr;
        }
        g.printProgress = true;
        if (count) *count = (int)h.size();
        if (hist)
            for (int i = 0; i < cap && i < (int)h.size(); i++) hist[i] = h[i];
    });
}

int gs_grid_vcycle(void* grid, double* residual)
{
    return guarded([&] {
        const double r = gs::HipSolver::vcycle(G(grid));
        if (residual) *residual = r;
    });
}

int gs_grid_jacobi(void* grid, int level, int sweeps)
{
    return guarded([&] { gs::HipSolver::jacobi(G(grid), (std::size_t)level, (std::size_t)sweeps); });
}

int gs_grid_residual_norm(void* grid, int level, double* norm)
{
    return guarded([&] {
        const double r = gs::HipSolver::compResidual(G(grid), (std::size_t)level, false, true);
        if (norm) *norm = r;
    });
}

int gs_grid_num_levels(void* grid) { return (int)G(grid).numLevels(); }

int gs_grid_level(void* grid, int level, gs_level* out)
{
    if (level < 0 || level >= (int)G(grid).numLevels() || !out) return 1;
    *out = G(grid).getLevel(level).geom;
    return 0;
}

double* gs_grid_field(void* grid, int level, int field)
{
    auto& g = G(grid);
    if (level < 0 || level >= (int)g.numLevels()) return nullptr;
    auto& L = g.getLevel(level);
    switch (field) {
    case 0: return L.v ? L.v.data() : nullptr;
    case 1: return L.restV ? L.restV.data() : nullptr;
    case 2: return L.newtonV ? L.newtonV.data() : nullptr;
    case 3: return L.f ? L.f.data() : nullptr;
    case 4: return L.r ? L.r.data() : nullptr;
    case 5: return (level == 0 && g.newtonF) ? g.newtonF.data() : nullptr;
    default: return nullptr;
    }
}

hipStream_t gs_grid_stream(void* grid) { return G(grid).stream(); }

static int copy_field(void* grid, int level, int field, double* host, const double* src_host)
{
    return guarded([&] {
        double* d = gs_grid_field(grid, level, field);
        if (!d) throw gs::Error("no such field on this level");
        const gs_level& L = G(grid).getLevel(level).geom;
        const size_t w = sizeof(double) * (size_t)(L.nx + 2), rows = (size_t)((L.ny + 2) * (L.nz + 2));
        const size_t pitch = sizeof(double) * (size_t)L.ldy;
        auto& g = G(grid);
        gs::check((int)hipStreamSynchronize(g.stream()), "hipStreamSynchronize");
        if (host)
            gs::check((int)hipMemcpy2D(host, w, d, pitch, w, rows, hipMemcpyDeviceToHost), "hipMemcpy2D");
        else
            gs::check((int)hipMemcpy2D(d, pitch, src_host, w, w, rows, hipMemcpyHostToDevice), "hipMemcpy2D");
    });
}

int gs_grid_download(void* grid, int level, int field, double* host)
{
    if (!host) return 1;
    return copy_field(grid, level, field, host, nullptr);
}

int gs_grid_upload(void* grid, int level, int field, const double* host)
{
    if (!host) return 1;
    return copy_field(grid, level, field, nullptr, host);
}

int gs_grid_sync(void* grid)
{
    return guarded([&] { gs::check((int)hipStreamSynchronize(G(grid).stream()), "hipStreamSynchronize"); });
}

int gs_grid_time_jacobi(void* grid, int level, int warmup, int sweeps, float* ms)
{
    return guarded([&] {
        auto& g = G(grid);
        gs::HipSolver::jacobi(g, (std::size_t)level, (std::size_t)warmup);
        hipEvent_t a, b;
        gs::check((int)hipEventCreate(&a), "hipEventCreate");
        gs::check((int)hipEventCreate(&b), "hipEventCreate");
        gs::check((int)hipEventRecord(a, g.stream()), "hipEventRecord");
        gs::HipSolver::jacobi(g, (std::size_t)level, (std::size_t)sweeps);
        gs::check((int)hipEventRecord(b, g.stream()), "hipEventRecord");
        gs::check((int)hipEventSynchronize(b), "hipEventSynchronize");
        float t = 0;
        gs::check((int)hipEventElapsedTime(&t, a, b), "hipEventElapsedTime");
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
        if (ms) *ms = t;
    });
}

int gs_grid_time_vcycles(void* grid, int cycles, double* ms, double* last_residual)
{
    return guarded([&] {
        auto& g = G(grid);
        gs::check((int)hipStreamSynchronize(g.stream()), "hipStreamSynchronize");
        const auto t0 = std::chrono::steady_clock::now();
        double r = 0;
        for (int c = 0; c < cycles; c++) r = gs::HipSolver::vcycle(g);
        const auto t1 = std::chrono::steady_clock::now();
        if (ms) *ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        if (last_residual) *last_residual = r;
    });
}

const char* gs_last_error(void) { return g_err.c_str(); }

} // extern "C"
