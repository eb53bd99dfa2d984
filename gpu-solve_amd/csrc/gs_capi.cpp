// gs_capi.cpp — extern "C" facade of the host driver (include/gpusolve_driver.h).
#include <algorithm>
#include <array>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <iostream>
#include <memory>
#include <string>
#include <thread>
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

// The opaque handle: the grid plus the communicator it runs on (owned here, not by the grid).
struct Handle {
    std::unique_ptr<gs::Comm> comm;
    std::unique_ptr<gs::HipGridData> grid;
};

gs::HipGridData& G(void* h) { return *static_cast<Handle*>(h)->grid; }

std::vector<std::array<int64_t, 3>> levelDims(const int64_t d[3])
{
    std::vector<std::array<int64_t, 3>> out;
    const int64_t mn = std::min(std::min(d[0], d[1]), d[2]);
    if (mn <= 0) return out;
    const int nlev = (int)std::floor(std::log((double)mn) / std::log(2.0)) + 1;
    std::array<int64_t, 3> c{d[0], d[1], d[2]};
    for (int l = 0; l < nlev; l++) {
        if (l) c = {c[0] / 2, c[1] / 2, c[2] / 2};
        out.push_back(c);
    }
    return out;
}

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
        auto* h = new Handle;
        h->grid = std::make_unique<gs::HipGridData>(toParams(p));
        return h;
    } catch (const std::exception& e) {
        g_err = e.what();
        return nullptr;
    }
}

void gs_grid_destroy(void* grid)
{
    auto* h = static_cast<Handle*>(grid);
    if (!h) return;
    h->grid.reset(); // before its communicator
    h->comm.reset();
    delete h;
}

int gs_grid_solve(void* grid, int print, double* hist, int cap, int* count)
{
    return guarded([&] {
        auto& g = G(grid);
        std::vector<double> h;
        g.printProgress = print != 0;
        if (g.mode == gs::GridParams::NEWTON) {
            gs::NewtonSolver::history = &h;
            try {
                gs::NewtonSolver::solve(g);
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

int gs_grid_level_fused(void* grid, int level)
{
    if (level < 0 || level >= (int)G(grid).numLevels()) return 0;
    return G(grid).getLevel(level).fusedPairs ? 1 : 0;
}

int gs_grid_level(void* grid, int level, gs_level* out)
{
    if (level < 0 || level >= (int)G(grid).numLevels() || !out) return 1;
    *out = G(grid).getLevel(level).geom;
    return 0;
}

// `writable`: the caller may write through the pointer (gs_grid_field, uploads), so the driver stops assuming
// anything about newtonV it derived earlier; reads (downloads, dumps) leave that state alone, so a rank that only
// reads its newtonV schedules exactly what the others do
static double* field_ptr(void* grid, int level, int field, bool writable)
{
    auto& g = G(grid);
    if (level < 0 || level >= (int)g.numLevels()) return nullptr;
    auto& L = g.getLevel(level);
    switch (field) {
    case 0: return L.v ? L.v.data() : nullptr;
    case 1: return L.restV ? L.restV.data() : nullptr;
    case 2:
        if (writable) g.newtonVTouched();
        return L.newtonV ? L.newtonV.data() : nullptr;
    case 3: return L.f ? L.f.data() : nullptr;
    case 4: return L.r ? L.r.data() : nullptr;
    case 5: return (level == 0 && g.newtonF) ? g.newtonF.data() : nullptr;
    default: return nullptr;
    }
}

double* gs_grid_field(void* grid, int level, int field) { return field_ptr(grid, level, field, true); }

hipStream_t gs_grid_stream(void* grid) { return G(grid).stream(); }

static int copy_field(void* grid, int level, int field, double* host, const double* src_host)
{
    return guarded([&] {
        double* d = field_ptr(grid, level, field, host == nullptr);
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

// Vector3::dump (src/cpu/Vector3.cpp:56-78): with a file, the header "Px Py Pz" then one line
// "x y z value" per padded point, x outermost and z innermost; without one (empty path or a file
// that cannot be opened) the same lines go to stdout, header omitted. Values use the iostream
// default format (6 significant digits, printf %g). Lines are formatted in parallel x-slabs and
// written in order.
int gs_dump_write(const double* host, int64_t px, int64_t py, int64_t pz, const char* path)
{
    return guarded([&] {
        if (!host || px < 0 || py < 0 || pz < 0) throw gs::Error("gs_dump_write: invalid argument");
        std::FILE* out = (path && *path) ? std::fopen(path, "w") : nullptr;
        std::FILE* dst = out ? out : stdout;
        if (out) std::fprintf(out, "%lld %lld %lld\n", (long long)px, (long long)py, (long long)pz);
        const int64_t nthreads = std::max<int64_t>(1, std::min<int64_t>(px, std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()))));
        const int64_t chunk = 8; // x-planes per task
        for (int64_t x0 = 0; x0 < px; x0 += chunk * nthreads) {
            std::vector<std::string> part((size_t)nthreads);
            std::vector<std::thread> th;
            for (int64_t t = 0; t < nthreads; t++)
                th.emplace_back([&, t] {
                    std::string& s = part[(size_t)t];
                    char buf[96];
                    for (int64_t x = x0 + t * chunk; x < std::min(px, x0 + (t + 1) * chunk); x++)
                        for (int64_t y = 0; y < py; y++)
                            for (int64_t z = 0; z < pz; z++) {
                                const int n = std::snprintf(buf, sizeof buf, "%lld %lld %lld %g\n", (long long)x,
                                                            (long long)y, (long long)z, host[x + px * (y + py * z)]);
                                s.append(buf, (size_t)n);
                            }
                });
            for (auto& t : th) t.join();
            for (auto& s : part) std::fwrite(s.data(), 1, s.size(), dst);
        }
        if (out) {
            if (std::fclose(out) != 0) throw gs::Error("gs_dump_write: write failed");
        } else {
            std::fflush(stdout);
        }
    });
}

int gs_grid_dump(void* grid, int level, int field, const char* path)
{
    if (level < 0 || level >= (int)G(grid).numLevels()) return guarded([] { throw gs::Error("no such level"); });
    const gs_level& L = G(grid).getLevel(level).geom;
    std::vector<double> host((size_t)((L.nx + 2) * (L.ny + 2) * (L.nz + 2)));
    const int rc = gs_grid_download(grid, level, field, host.data());
    if (rc) return rc;
    return gs_dump_write(host.data(), L.nx + 2, L.ny + 2, L.nz + 2, path);
}

int gs_grid_metrics(void* grid, char* line, int cap, double* level_ms, int levels_cap)
{
    return guarded([&] {
        auto& g = G(grid);
        if (!g.clock.on) throw gs::Error("metrics are off (set GS_METRICS=1 before creating the grid)");
        const std::string s = gs::metricsLine(g);
        if (line && cap > 0) {
            std::strncpy(line, s.c_str(), (size_t)cap - 1);
            line[cap - 1] = 0;
        }
        for (int l = 0; level_ms && l < levels_cap && l < (int)g.clock.levelMs.size(); l++)
            level_ms[l] = g.clock.cycles ? g.clock.levelMs[l] / g.clock.cycles : 0.0;
    });
}

int gs_grid_sync(void* grid)
{
    return guarded([&] { G(grid).sync(); });
}

int gs_grid_comm_stats(void* grid, double* halo_host_ms, int64_t* halo_calls)
{
    return guarded([&] {
        const auto& g = G(grid);
        if (halo_host_ms) *halo_host_ms = g.haloHostMs;
        if (halo_calls) *halo_calls = g.haloCalls;
    });
}

int gs_grid_comm_stats_max(void* grid, double* halo_host_max_ms)
{
    return guarded([&] {
        if (halo_host_max_ms) *halo_host_max_ms = G(grid).haloHostMaxMs;
    });
}

int gs_grid_comm_ctas(void* grid)
{
    if (!grid) return -1;
    const auto* h = static_cast<Handle*>(grid);
    return h->comm ? h->comm->ctas() : -1;
}

int gs_rccl_channels_per_peer_hint(int ctas) { return gs::rcclChannelsPerPeerHint(ctas); }

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
        // the solve loop's steady state: speculative closing norms (HipSolver::solve)
        int pending = 0;
        if (gs::HipSolver::speculationEnabled(g)) gs::HipSolver::speculativeSweep(g, &pending);
        gs::check((int)hipStreamSynchronize(g.stream()), "hipStreamSynchronize");
        const auto t0 = std::chrono::steady_clock::now();
        double r = 0;
        gs::HipSolver::runCycles(g, &pending, (std::size_t)std::max(cycles, 0), [&](std::size_t, double res) {
            r = res;
            return false;
        }); // (a speculative sweep left in vAlt is dropped: v stays the last cycle's result)
        const auto t1 = std::chrono::steady_clock::now();
        if (ms) *ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        if (last_residual) *last_residual = r;
    });
}

int gs_zslab_plan(const int64_t dims[3], int nranks, int64_t min_points, int max_levels, int* distributed,
                  int64_t* lo, int64_t* hi)
{
    const auto ld = levelDims(dims);
    if (ld.empty() || nranks < 1) return 0;
    std::vector<int64_t> nz, pts;
    for (auto& d : ld) {
        nz.push_back(d[2]);
        pts.push_back(d[0] * d[1] * d[2]);
    }
    if (min_points < 0) {
        const char* e = std::getenv("GS_ZSLAB_MIN_POINTS");
        min_points = e ? std::atoll(e) : 32768;
    }
    const gs::SlabPlan plan = gs::planZSlabs(nz, pts, nranks, min_points);
    for (int l = 0; l < (int)ld.size() && l < max_levels; l++) {
        if (distributed) distributed[l] = plan.distributed[l];
        for (int r = 0; r < nranks; r++) {
            if (lo) lo[l * nranks + r] = plan.lo[l][r];
            if (hi) hi[l * nranks + r] = plan.hi[l][r];
        }
    }
    return (int)ld.size();
}

int gs_zslab_schedule(const gs_params* p, int nranks, int rank, int64_t min_points, char* buf, int64_t cap,
                      int64_t* len)
{
    return guarded([&] {
        if (!p || nranks < 1 || rank < 0 || rank >= nranks) throw gs::Error("gs_zslab_schedule: bad arguments");
        std::vector<std::string> ops;
        {
            auto comm = gs::makeTraceComm(rank, nranks);
            gs::HipGridData g(toParams(p), comm.get(), min_points, &ops);
            g.printProgress = false;
            // the solve's residuals are read (as GpuSolve-hip prints them): every closing norm is in the schedule
            std::vector<double> hist;
            gs::NewtonSolver::history = &hist;
            gs::HipSolver::history = &hist;
            try {
                if (g.mode == gs::GridParams::NEWTON) gs::NewtonSolver::solve(g);
                else gs::HipSolver::solve(g);
            } catch (...) {
                gs::NewtonSolver::history = nullptr;
                gs::HipSolver::history = nullptr;
                throw;
            }
            gs::NewtonSolver::history = nullptr;
            gs::HipSolver::history = nullptr;
        }
        std::string text;
        for (const auto& o : ops) text += o + "\n";
        if (len) *len = (int64_t)text.size();
        if (buf && cap > 0) {
            const std::size_t n = std::min<std::size_t>(text.size(), (std::size_t)cap - 1);
            std::memcpy(buf, text.data(), n);
            buf[n] = 0;
        }
    });
}

int gs_rccl_unique_id(unsigned char uid[128])
{
    return guarded([&] { gs::rcclUniqueId(uid); });
}

void* gs_grid_create_rccl(const gs_params* p, int rank, int nranks, const unsigned char uid[128])
{
    return gs_grid_create_rccl_ctas(p, rank, nranks, uid, -1);
}

void* gs_grid_create_rccl_ctas(const gs_params* p, int rank, int nranks, const unsigned char uid[128], int ctas)
{
    if (!p || !uid || rank < 0 || rank >= nranks || ctas < -1) {
        g_err = "bad arguments";
        return nullptr;
    }
    try {
        auto* h = new Handle;
        try {
            h->comm = gs::makeRcclComm(rank, nranks, uid, ctas);
            h->grid = std::make_unique<gs::HipGridData>(toParams(p), h->comm.get());
        } catch (...) {
            gs_grid_destroy(h);
            throw;
        }
        return h;
    } catch (const std::exception& e) {
        g_err = e.what();
        return nullptr;
    }
}

int gs_uid_publish(const char* path, const unsigned char uid[128])
{
    if (!path || !uid) {
        g_err = "bad arguments";
        return 1;
    }
    try {
        gs::publishUid(path, uid);
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return 1;
    }
}

int gs_uid_default_path(char* buf, int cap)
{
    const std::string p = gs::uidPath();
    if (buf && cap > 0) {
        std::strncpy(buf, p.c_str(), (size_t)cap - 1);
        buf[cap - 1] = 0;
    }
    return (int)p.size();
}

int gs_uid_await(const char* path, double timeout_s, unsigned char uid[128])
{
    if (!path || !uid) {
        g_err = "bad arguments";
        return 1;
    }
    try {
        gs::awaitUid(path, timeout_s, uid);
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return 1;
    }
}

int gs_zslab_loopback_run(const gs_params* p, int nranks, int64_t min_points, int sweeps, int solve, double* hist,
                          int cap, int* count, double* v_host)
{
    if (!p || nranks < 1) return 1;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        g_err = "no HIP device";
        return 1;
    }
    auto hub = gs::makeLoopbackHub(nranks);
    std::vector<std::string> errs(nranks);
    std::vector<double> h0;
    const gs::GridParams params = toParams(p);
    // test hook: GS_LOOPBACK_TOUCH_NEWTONV=r marks rank r's newtonV as handed out before the solve (what
    // gs_grid_field does), so that rank alone loses the zero-newtonV shortcut unless the solver agrees on it
    const char* touchEnv = std::getenv("GS_LOOPBACK_TOUCH_NEWTONV");
    const int touchRank = touchEnv && *touchEnv ? std::atoi(touchEnv) : -1;
    auto body = [&](int r) {
        try {
            gs::check((int)hipSetDevice(dev), "hipSetDevice");
            auto comm = gs::makeLoopbackComm(hub, r);
            gs::HipGridData g(params, comm.get(), min_points);
            gs::HipSolver::jacobi(g, 0, (std::size_t)sweeps);
            if (r == touchRank) g.newtonVTouched();
            if (solve) {
                g.printProgress = false;
                std::vector<double> h;
                if (g.mode == gs::GridParams::NEWTON) {
                    gs::NewtonSolver::history = &h;
                    gs::NewtonSolver::solve(g);
                    gs::NewtonSolver::history = nullptr;
                } else {
                    gs::HipSolver::history = &h;
                    gs::HipSolver::solve(g);
                    gs::HipSolver::history = nullptr;
                }
                if (r == 0) h0 = h;
            }
            gs::check((int)hipStreamSynchronize(g.stream()), "hipStreamSynchronize");
            if (v_host) {
                auto& L = g.getLevel(0);
                const gs_level& G0 = L.geom;
                const size_t w = sizeof(double) * (size_t)(G0.nx + 2);
                double* dst = v_host + (size_t)L.lo * (size_t)((G0.ny + 2) * (G0.nx + 2));
                gs::check((int)hipMemcpy2D(dst, w, L.v.data() + G0.ldz, sizeof(double) * (size_t)G0.ldy, w,
                                           (size_t)((G0.ny + 2) * G0.nz), hipMemcpyDeviceToHost),
                          "hipMemcpy2D");
            }
        } catch (const std::exception& e) {
            errs[r] = e.what();
            // the other ranks may be parked in (or heading for) a hub barrier this rank will never
            // reach: wake them, and make every later barrier throw, so all threads unwind and join
            gs::abortLoopbackHub(*hub, e.what());
        }
    };
    std::vector<std::thread> th;
    for (int r = 0; r < nranks; r++) th.emplace_back(body, r);
    for (auto& t : th) t.join();
    const std::string first = gs::loopbackHubError(*hub); // the failure that aborted the others
    if (!first.empty()) {
        g_err = first;
        return 1;
    }
    for (auto& e : errs)
        if (!e.empty()) {
            g_err = e;
            return 1;
        }
    if (count) *count = (int)h0.size();
    if (hist)
        for (int i = 0; i < cap && i < (int)h0.size(); i++) hist[i] = h0[i];
    return 0;
}

int gs_debug_bounded_wait(int scenario, int k, double timeout_s, char* msg, int cap)
{
    std::string err;
    const int rc = gs::debugBoundedWait(scenario, k, timeout_s, &err);
    if (msg && cap > 0) {
        std::strncpy(msg, err.c_str(), (size_t)cap - 1);
        msg[cap - 1] = 0;
    }
    return rc;
}

int gs_debug_loopback_abort(int nranks, int failing_rank)
{
    return gs::debugLoopbackAbort(nranks, failing_rank, &g_err);
}

const char* gs_last_error(void) { return g_err.c_str(); }

} // extern "C"
