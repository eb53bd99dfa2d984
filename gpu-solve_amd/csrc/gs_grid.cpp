// gs_grid.cpp — HipGridData, HipSolver, NewtonSolver (see gs_grid.hpp).
#include "gs_grid.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <utility>

#include <hip/hip_runtime.h>

#include "gpusolve_driver.h"

namespace gs {

void check(int code, const char* what)
{
    if (code != 0) throw Error(std::string(what) + ": " + gs_strerror(code));
}

// ---------------------------------------------------------------------------------------------
DeviceField::DeviceField(int64_t nx, int64_t ny, int64_t nz, hipStream_t s, bool dry) : dry_(dry)
{
    int64_t origin = 0;
    check(gs_field_layout(nx, ny, nz, &ldy_, &ldz_, &alloc_, &origin), "gs_field_layout");
    span_ = ldz_ * (nz + 2);
    if (dry) return;
    void* p = nullptr;
    check((int)hipMalloc(&p, sizeof(double) * alloc_), "hipMalloc");
    base_ = static_cast<double*>(p);
    origin_ = base_ + origin;
    span_ = ldz_ * (nz + 2);
    zero(s);
}

DeviceField::~DeviceField()
{
    if (base_) (void)hipFree(base_);
}

DeviceField& DeviceField::operator=(DeviceField&& o) noexcept
{
    if (this != &o) {
        if (base_) (void)hipFree(base_);
        base_ = std::exchange(o.base_, nullptr);
        origin_ = std::exchange(o.origin_, nullptr);
        ldy_ = o.ldy_;
        ldz_ = o.ldz_;
        span_ = o.span_;
        alloc_ = o.alloc_;
        dry_ = o.dry_;
    }
    return *this;
}

bool HipGridData::allRanks(bool flag)
{
    if (trace || !comm_ || comm_->size() <= 1) return flag;
    const hipStream_t s = stream();
    const double on = flag ? 1.0 : 0.0;
    std::vector<double> all((std::size_t)comm_->size(), 0.0);
    check((int)hipMemcpyAsync(dNorm_, &on, sizeof(double), hipMemcpyHostToDevice, s), "hipMemcpyAsync");
    comm_->allgather1(dNorm_, dRankSums_, s);
    check((int)hipMemcpyAsync(all.data(), dRankSums_, sizeof(double) * all.size(), hipMemcpyDeviceToHost, s),
          "hipMemcpyAsync");
    comm_->sync(s);
    for (const double a : all) flag = flag && a != 0.0;
    return flag;
}

void DeviceField::zero(hipStream_t s)
{
    if (base_) check((int)hipMemsetAsync(base_, 0, sizeof(double) * alloc_, s), "hipMemsetAsync");
}

void DeviceField::swap(DeviceField& o) noexcept
{
    std::swap(base_, o.base_);
    std::swap(origin_, o.origin_);
    std::swap(ldy_, o.ldy_);
    std::swap(ldz_, o.ldz_);
    std::swap(span_, o.span_);
    std::swap(alloc_, o.alloc_);
    std::swap(dry_, o.dry_);
}

DeviceBuf::~DeviceBuf()
{
    if (p_) (void)hipFree(p_);
}

double* DeviceBuf::get(int64_t elems)
{
    if (elems <= n_) return p_;
    if (p_) check((int)hipFree(p_), "hipFree");
    p_ = nullptr;
    n_ = 0;
    void* q = nullptr;
    check((int)hipMalloc(&q, sizeof(double) * (size_t)elems), "hipMalloc(workspace)");
    p_ = static_cast<double*>(q);
    n_ = elems;
    return p_;
}

StreamGuard::StreamGuard(bool create, bool high)
{
    if (!create) return;
    int least = 0, greatest = 0;
    if (high && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
        check((int)hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest), "hipStreamCreateWithPriority");
    else
        check((int)hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
}
StreamGuard::~StreamGuard()
{
    if (s) (void)hipStreamDestroy(s);
}

// ---------------------------------------------------------------------------------------------
void LevelClock::mark(hipStream_t s, int level, bool begin)
{
    if (!on) return;
    const std::size_t k = segLevel.size();
    if (begin) {
        if (ev.size() < 2 * (k + 1)) {
            for (int j = 0; j < 2; j++) {
                hipEvent_t e = nullptr;
                check((int)hipEventCreate(&e), "hipEventCreate");
                ev.push_back(e);
            }
        }
        segLevel.push_back(level);
        check((int)hipEventRecord(ev[2 * k], s), "hipEventRecord");
    } else if (k > 0) {
        check((int)hipEventRecord(ev[2 * k - 1], s), "hipEventRecord");
    }
}

void LevelClock::collect()
{
    if (!on) return;
    for (std::size_t k = 0; k < segLevel.size(); k++) {
        float ms = 0.f;
        check((int)hipEventSynchronize(ev[2 * k + 1]), "hipEventSynchronize");
        check((int)hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]), "hipEventElapsedTime");
        const std::size_t l = (std::size_t)segLevel[k];
        if (levelMs.size() <= l) levelMs.resize(l + 1, 0.0);
        levelMs[l] += ms;
    }
    segLevel.clear();
}

LevelClock::~LevelClock()
{
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
}

int64_t proWsElems(const HipGridData& g, std::size_t l); // below

// ---------------------------------------------------------------------------------------------
// Level hierarchy: L = floor(log2(min dim)) + 1, dims halve per level, h_l = 1/(ny_l+1)
// (src/cpu/CpuGridData.cpp:19-41). Fields a mode never touches are not allocated.
HipGridData::HipGridData(const GridParams& grid, Comm* comm, int64_t agglomeratePoints,
                         std::vector<std::string>* traceLog)
    : GridParams(grid), trace(traceLog), comm_(comm), stream_(traceLog == nullptr),
      // the exchange path at high priority: when the interior sweep's blocks retire, the dispatcher
      // hands the freed CUs to the boundary planes and the ghost exchange first
      commStream_(traceLog == nullptr, true), bndStream_(traceLog == nullptr && comm != nullptr && comm->size() > 1, true)
{
    const bool dry = traceLog != nullptr;
    const std::size_t mn = std::min(std::min(gridDim[0], gridDim[1]), gridDim[2]);
    if (mn == 0) throw Error("grid dimensions must be positive");
    const int nlev = (int)std::floor(std::log((double)mn) / std::log(2.0)) + 1;
    levels_.resize(nlev);
    for (int i = 0; i < 7; i++) {
        stencilAbi.s[i] = stencil.values[i];
        stencilAbi.ox[i] = stencil.getXOffset(i);
        stencilAbi.oy[i] = stencil.getYOffset(i);
        stencilAbi.oz[i] = stencil.getZOffset(i);
    }
    {
        auto on = [](const char* name) { return std::getenv(name) != nullptr; };
        sw.fusedSweeps = !on("GS_NO_FUSED_SWEEPS");
        sw.speculation = !on("GS_NO_SPECULATION");
        sw.fusedProlong = !on("GS_NO_FUSED_PROLONG");
        sw.fusedRR = !on("GS_NO_FUSED_RR");
        sw.zeroGuess = !on("GS_NO_ZERO_GUESS");
        sw.pipeline = !on("GS_NO_PIPELINE");
        sw.newtonFusedUpdate = !on("GS_NO_NEWTON_FUSED_UPDATE");
        sw.newtonB = !on("GS_NO_NEWTON_B");
        if (const char* e = std::getenv("GS_NEWTON_B_FUSED")) sw.newtonBFused = std::atoi(e) != 0;
        sw.newtonG = !on("GS_NO_NEWTON_G");
        if (const char* e = std::getenv("GS_NEWTON_PRO_POINTS")) sw.newtonProPoints = std::strtoll(e, nullptr, 10);
        if (const char* e = std::getenv("GS_TILE_POINTS")) sw.tilePoints = std::strtoll(e, nullptr, 10);
        if (const char* e = std::getenv("GS_HALO_ORDER")) sw.haloOrder = std::atoi(e);
    }
    std::vector<int64_t> nzs, pts;
    for (int l = 0; l < nlev; l++) {
        LevelData& L = levels_[l];
        L.levelDim = l == 0 ? gridDim
                            : std::array<std::size_t, 3>{levels_[l - 1].levelDim[0] / 2, levels_[l - 1].levelDim[1] / 2,
                                                         levels_[l - 1].levelDim[2] / 2};
        nzs.push_back((int64_t)L.levelDim[2]);
        pts.push_back((int64_t)(L.levelDim[0] * L.levelDim[1] * L.levelDim[2]));
    }
    if (agglomeratePoints < 0) {
        const char* e = std::getenv("GS_ZSLAB_MIN_POINTS");
        agglomeratePoints = e ? std::atoll(e) : 32768;
    }
    const SlabPlan plan = planZSlabs(nzs, pts, nranks(), agglomeratePoints);

    const hipStream_t s = stream_.s;
    int64_t maxParts = 1;
    for (int l = 0; l < nlev; l++) {
        LevelData& L = levels_[l];
        const int64_t nx = (int64_t)L.levelDim[0], ny = (int64_t)L.levelDim[1];
        L.distributed = plan.distributed[l];
        L.ranksLo = plan.lo[l];
        L.ranksHi = plan.hi[l];
        if (L.distributed) {
            L.lo = plan.lo[l][rank()];
            L.hi = plan.hi[l][rank()];
        } else {
            L.lo = 1;
            L.hi = (int64_t)L.levelDim[2];
        }
        const int64_t nz = L.hi - L.lo + 1;
        L.h = 1.0 / (L.levelDim[1] + 1);
        L.v = DeviceField(nx, ny, nz, s, dry);
        L.vAlt = DeviceField(nx, ny, nz, s, dry);
        L.f = DeviceField(nx, ny, nz, s, dry);
        if (l + 1 < nlev) L.r = DeviceField(nx, ny, nz, s, dry); // restriction source
        if (mode == NONLINEAR && l > 0) L.restV = DeviceField(nx, ny, nz, s, dry);
        if (mode == NEWTON) L.newtonV = DeviceField(nx, ny, nz, s, dry);
        if (mode == NEWTON && sw.newtonB && dry) L.bfac = DeviceField(nx, ny, nz, s, dry); // (else: below)
        if (mode == NEWTON && l == 1 && nlev >= 3 && !L.distributed) L.newtonVNext = DeviceField(nx, ny, nz, s, dry);
        L.geom = gs_level{nx, ny, nz, L.v.ldy(), L.v.ldz(), L.lo - 1, L.h};
        maxParts = std::max(maxParts, gs_residual_num_partials(&stencilAbi, &L.geom));
        maxParts = std::max(maxParts, gs_jacobi_sweep2_num_partials(&stencilAbi, &L.geom, (int)mode));
        L.minPlanes = nz;
        if (L.distributed)
            for (int q = 0; q < nranks(); q++) L.minPlanes = std::min(L.minPlanes, L.ranksHi[q] - L.ranksLo[q] + 1);
        // rank-uniform on a Z-slab level (the smoothing schedule decides the ghost exchanges): judged
        // on the thinnest slab, as the kernel's fill count grows with the plane count
        gs_level thin = L.geom;
        thin.nz = L.minPlanes;
        L.fusedPairs = sw.fusedSweeps && gs_jacobi_sweep2_supported_mode(&stencilAbi, &thin, (int)mode) == 2 &&
                       (!L.distributed || L.minPlanes >= 2);
        L.tiled = !L.distributed && pts[l] <= sw.tilePoints &&
                  gs_tiled_supported(&stencilAbi, &L.geom, (int)mode) != 0;
    }
    // The coarse end of the V-cycle runs as one gs_coarse_cycle launch from the first level of at
    // most GS_COARSE_POINTS points that is not Z-slab partitioned; 0 = off. Default 512 = 8^3: a 16^3
    // level costs 42 us inside the one workgroup (a single CU's L2 bandwidth: ~6 us per operator)
    // against 30 us as six chip-wide launches; from 8^3 down the launch wins (tools/ab_coarse.sh).
    coarseFrom = levels_.size();
    {
        const char* e = std::getenv("GS_COARSE_POINTS");
        const int64_t thr = e ? std::atoll(e) : 512;
        if (thr > 0 && preSmoothing + postSmoothing < (1u << 20))
            for (int l = nlev - 1; l >= 1; l--) {
                if (levels_[l].distributed || pts[l] > thr || nlev - l > gs_coarse_cycle_max_levels()) break;
                coarseFrom = (std::size_t)l;
            }
    }
    if (mode == NEWTON) newtonF = DeviceField(levels_[0].geom.nx, levels_[0].geom.ny, levels_[0].geom.nz, s, dry);
    newtonVZero_ = mode == NEWTON; // (every field is created zero-filled)
    {
        const char* e = std::getenv("GS_METRICS");
        clock.on = !dry && e && *e && *e != '0';
        clock.levelMs.assign(nlev, 0.0);
    }
    if (dry) {
        dryParts_.assign(16, 0.0); // the partial-sum pointers the solvers pass mark normed launches
        partials_ = dryParts_.data();
        rec("rhs", {{"L", 0}}, "f");
        halo(levels_[0], levels_[0].f, s);
        return;
    }
    // the overlapped sweep splits a level into 3 launches, each with its own partials region
    maxParts = 2 * maxParts + 4096;
    check((int)hipMalloc((void**)&partials_, sizeof(double) * maxParts), "hipMalloc(partials)");
    check((int)hipMalloc((void**)&dNorm_, sizeof(double)), "hipMalloc(norm)");
    check((int)hipMalloc((void**)&dRankSums_, sizeof(double) * nranks()), "hipMalloc(rank sums)");
    // the final norm goes straight from the finishing kernel to this pinned word (no D2H copy launch)
    check((int)hipHostMalloc((void**)&hNorm_, sizeof(double), hipHostMallocMapped | hipHostMallocCoherent),
          "hipHostMalloc");
    check((int)hipHostGetDevicePointer((void**)&hNormDev_, hNorm_, 0), "hipHostGetDevicePointer");
    check((int)hipEventCreateWithFlags(&evA_, hipEventDisableTiming), "hipEventCreate");
    check((int)hipEventCreateWithFlags(&evB_, hipEventDisableTiming), "hipEventCreate");
    check((int)hipEventCreateWithFlags(&evC_, hipEventDisableTiming), "hipEventCreate");
    for (auto& e : evBnd_) check((int)hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    check((int)hipEventCreateWithFlags(&evNorm_, hipEventDisableTiming), "hipEventCreate");
    // level-0 right-hand side on the device (src/cpu/CpuGridData.cpp:44-78), h = 1/(Y+1) (main.cpp:84);
    // a slab evaluates it at its global plane indices (geom.z0)
    check(gs_rhs_init(&levels_[0].geom, levels_[0].f.data(), (int)mode, 1.0 / (gridDim[1] + 1), gamma, s),
          "gs_rhs_init");
    halo(levels_[0], levels_[0].f, s); // the fused pair's first sweep reads f on a ghost plane
    // GS_METRICS is read by each process, but the per-level clock changes the collective schedule (no
    // pipelined cycles; the last closing norm is kept): a distributed grid runs it only if EVERY rank has it
    // on, so that all ranks issue the same exchanges and collectives
    clock.on = allRanks(clock.on);
    // GS_NEWTON_B's factor fields: one more level-sized array per NEWTON level (~8.6 GB at 1023^3). If they do not
    // fit, the grid runs the reference-expression inner solves (mode 2, GS_NO_NEWTON_B) instead of failing; the
    // choice is agreed across ranks (it changes which kernels run, never the exchanges, but stays uniform)
    if (mode == NEWTON && sw.newtonB) {
        bool ok = true;
        try {
            for (auto& L : levels_) L.bfac = DeviceField(L.geom.nx, L.geom.ny, L.geom.nz, s, dry);
        } catch (const Error&) {
            ok = false;
            (void)hipGetLastError(); // (the failed hipMalloc's sticky error)
        }
        if (!allRanks(ok)) {
            sw.newtonB = false;
            for (auto& L : levels_) L.bfac = DeviceField();
        }
    }
    // the fused prolongation pair's edge-column workspaces (column-block rows), one per stream, at their
    // largest size now: proPlanes never reallocates them
    for (int l = 0; l + 1 < nlev; l++) {
        const int64_t need = proWsElems(*this, (std::size_t)l);
        if (need <= 0) continue;
        levels_[l].proWs[0].get(need);
        if (bndStream_.s) levels_[l].proWs[1].get(need);
    }
    check((int)hipStreamSynchronize(s), "hipStreamSynchronize");
}

HipGridData::~HipGridData()
{
    if (stream_.s) (void)hipStreamSynchronize(stream_.s);
    if (commStream_.s) (void)hipStreamSynchronize(commStream_.s);
    if (bndStream_.s) (void)hipStreamSynchronize(bndStream_.s);
    if (partials_ && !trace) (void)hipFree(partials_);
    if (dNorm_) (void)hipFree(dNorm_);
    if (dRankSums_) (void)hipFree(dRankSums_);
    if (hNorm_) (void)hipHostFree(hNorm_);
    if (evA_) (void)hipEventDestroy(evA_);
    if (evB_) (void)hipEventDestroy(evB_);
    if (evC_) (void)hipEventDestroy(evC_);
    for (auto e : evBnd_)
        if (e) (void)hipEventDestroy(e);
    if (evNorm_) (void)hipEventDestroy(evNorm_);
}

void HipGridData::rec(const char* op, std::initializer_list<std::pair<const char*, long long>> kv, const char* field)
{
    std::string line = op;
    if (field) line += std::string(" field=") + field;
    for (const auto& p : kv) line += " " + std::string(p.first) + "=" + std::to_string(p.second);
    trace->push_back(line);
}

const char* HipGridData::fieldName(const LevelData& L, const DeviceField& f)
{
    if (&f == &L.v) return "v";
    if (&f == &L.vAlt) return "vAlt";
    if (&f == &L.f) return "f";
    if (&f == &L.r) return "r";
    if (&f == &L.restV) return "restV";
    if (&f == &L.newtonV) return "newtonV";
    if (&f == &L.bfac) return "bfac";
    return "?";
}

// Trace mode has no device: the norms are placeholders (1.0, never a stop), except that
// GS_TRACE_STOP_AFTER=k makes the norm closing cycle k read 0.0, so that the loop stops there and the
// schedule records an early stop (tests replay it: the undo of the overlapped next cycle's adoption).
double HipGridData::traceNorm()
{
    const char* e = std::getenv("GS_TRACE_STOP_AFTER"); // read per call: tests switch it
    const long stopAfter = e ? std::strtol(e, nullptr, 10) : -1;
    const long read = traceNorms_++; // 0: the initial norm, i + 1: cycle i's closing norm
    return (stopAfter >= 0 && read == stopAfter + 1) ? 0.0 : 1.0;
}

double HipGridData::readNorm()
{
    if (trace) return traceNorm();
    sync();
    return *(volatile double*)hNorm_;
}

void HipGridData::readNormBegin()
{
    if (trace) return;
    check((int)hipEventRecord(evNorm_, stream_.s), "hipEventRecord");
}

double HipGridData::readNormEnd()
{
    if (trace) return traceNorm();
    // distributed: a bounded wait that also polls the communicator's error state (gs_comm.hpp)
    if (comm_ && comm_->size() > 1) comm_->syncEvent(evNorm_);
    else check((int)hipEventSynchronize(evNorm_), "hipEventSynchronize");
    return *(volatile double*)hNorm_;
}

void HipGridData::sync()
{
    if (trace) return;
    // distributed: a bounded wait that also polls the communicator's error state (gs_comm.hpp)
    if (comm_ && comm_->size() > 1) comm_->sync(stream_.s);
    else check((int)hipStreamSynchronize(stream_.s), "hipStreamSynchronize");
}

void HipGridData::halo(LevelData& L, DeviceField& fld, hipStream_t s, int depth)
{
    if (!(L.distributed && nranks() > 1)) return;
    if (trace) {
        rec("halo", {{"L", (long long)levelIndex(L)}, {"depth", depth}}, fieldName(L, fld));
        return;
    }
    haloSettle(); // (an exchange of the pipelined sequence is settled before anything else is issued)
    // host cost of issuing + settling the exchange (RCCL: group start/end and the async-error poll)
    const auto t0 = std::chrono::steady_clock::now();
    comm_->halo(fld.data(), fld.ldz(), L.geom.nz, depth, s);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    haloHostMs += ms;
    haloHostMaxMs = std::max(haloHostMaxMs, ms);
    haloCalls++;
}

void HipGridData::haloIssue(LevelData& L, DeviceField& fld, hipStream_t s, int depth)
{
    if (!(L.distributed && nranks() > 1)) return;
    if (trace) {
        rec("halo", {{"L", (long long)levelIndex(L)}, {"depth", depth}}, fieldName(L, fld));
        return;
    }
    haloSettle();
    const auto t0 = std::chrono::steady_clock::now();
    comm_->haloIssue(fld.data(), fld.ldz(), L.geom.nz, depth, s);
    haloCurMs_ = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    haloPending_ = true;
}

bool HipGridData::haloReady()
{
    if (trace) return sw.haloOrder != 1;
    if (!haloPending_) return sw.haloOrder != 1;
    const auto t0 = std::chrono::steady_clock::now();
    const bool ok = comm_->haloReady();
    haloCurMs_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (sw.haloOrder == 1) return false;
    return sw.haloOrder == 2 || ok;
}

void HipGridData::haloSettle()
{
    if (!haloPending_) return;
    const auto t0 = std::chrono::steady_clock::now();
    comm_->haloSettle();
    haloCurMs_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    haloPending_ = false;
    haloHostMs += haloCurMs_;
    haloHostMaxMs = std::max(haloHostMaxMs, haloCurMs_);
    haloCalls++;
}

void HipGridData::gather(LevelData& L, DeviceField& fld)
{
    if (trace) rec("gather", {{"L", (long long)levelIndex(L)}}, fieldName(L, fld));
    else comm_->gatherPlanes(fld.data(), fld.ldz(), L.ranksLo, L.ranksHi, stream_.s);
}

gs_level HipGridData::ownedGeom(const LevelData& L, int64_t* off) const
{
    gs_level g = L.geom;
    *off = 0;
    const std::size_t l = &L - levels_.data();
    const bool transition = l > 0 && !L.distributed && levels_[l - 1].distributed;
    if (transition) {
        const int64_t lo = L.ranksLo[rank()], hi = L.ranksHi[rank()];
        g.nz = std::max<int64_t>(0, hi - lo + 1);
        g.z0 = lo - 1;
        *off = (lo - 1) * L.geom.ldz;
    }
    return g;
}

// ---------------------------------------------------------------------------------------------
thread_local std::vector<double>* HipSolver::history = nullptr;
thread_local std::vector<double>* NewtonSolver::history = nullptr;

namespace {

// one fused sweep over local planes [z1, z2] of level L: reads L.v, writes L.vAlt; with partials,
// also the per-block r^2 sums of the input's residual. Returns the partial count written.
int64_t sweepPlanes(HipGridData& g, HipGridData::LevelData& L, int64_t z1, int64_t z2, hipStream_t s,
                    double* partials = nullptr)
{
    if (z2 < z1) return 0;
    gs_level sub = L.geom;
    sub.nz = z2 - z1 + 1;
    sub.z0 += z1 - 1;
    const int64_t off = (z1 - 1) * L.geom.ldz;
    if (g.trace) {
        g.rec("sweep", {{"L", (long long)g.levelIndex(L)}, {"z1", z1}, {"z2", z2}, {"vzero", L.vZero}, {"norm", partials != nullptr}});
        return partials ? 1 : 0;
    }
    check(gs_jacobi_sweep_norm(&g.stencilAbi, &sub, g.kmode(), g.omega, g.gamma, L.vZero ? nullptr : L.v.data() + off,
                               L.vAlt.data() + off, L.f.data() + off, g.wOf(L) ? g.wOf(L) + off : nullptr,
                               partials, s),
          "gs_jacobi_sweep");
    return partials ? gs_residual_num_partials(&g.stencilAbi, &sub) : 0;
}

// two fused sweeps over local planes [z1, z2]: reads L.v (two ghost planes deep where a side is an
// internal boundary), writes L.vAlt; with partials, also the per-block r^2 sums of the input's
// residual. Returns the partial count written.
int64_t pairPlanes(HipGridData& g, HipGridData::LevelData& L, int64_t z1, int64_t z2, hipStream_t s,
                   double* partials = nullptr)
{
    if (z2 < z1) return 0;
    gs_level sub = L.geom;
    sub.nz = z2 - z1 + 1;
    sub.z0 += z1 - 1;
    const int64_t off = (z1 - 1) * L.geom.ldz;
    const bool dist = L.distributed && g.nranks() > 1;
    const int zlo = z1 > 1 || (dist && g.rank() > 0);
    const int zhi = z2 < L.geom.nz || (dist && g.rank() + 1 < g.nranks());
    if (g.trace) {
        g.rec("pair", {{"L", (long long)g.levelIndex(L)}, {"z1", z1}, {"z2", z2}, {"zlo", zlo}, {"zhi", zhi},
                       {"vzero", L.vZero}, {"norm", partials != nullptr}});
        return partials ? 1 : 0;
    }
    check(gs_jacobi_sweep2_norm(&g.stencilAbi, &sub, g.kmode(), g.omega, g.gamma, L.vZero ? nullptr : L.v.data() + off,
                                L.vAlt.data() + off, L.f.data() + off, g.wOf(L) ? g.wOf(L) + off : nullptr,
                                zlo, zhi, partials, s),
          "gs_jacobi_sweep2");
    return partials ? gs_jacobi_sweep2_num_partials(&g.stencilAbi, &sub, (int)g.mode) : 0;
}

// The first post-smoothing pair of v^h + P v^2h (gs_jacobi_sweep2_prolong) on planes z1..z2 of F
// into F.vAlt. Every plane range starts on an odd plane (the kernel's parities are global ones) and
// ends two planes below the level's top or on it: the planes past an internal range end are
// interior planes (or a neighbour's ghost copies), which the kernel corrects as it reads them.
void proPlanes(HipGridData& g, HipGridData::LevelData& F, HipGridData::LevelData& C, int64_t z1, int64_t z2,
               hipStream_t s)
{
    if (z2 < z1) return;
    gs_level sub = F.geom;
    sub.nz = z2 - z1 + 1;
    sub.z0 += z1 - 1;
    const int64_t off = (z1 - 1) * F.geom.ldz;
    const bool dist = F.distributed && g.nranks() > 1;
    const int zlo = z1 > 1 || (dist && g.rank() > 0);
    const int zhi = z2 < F.geom.nz || (dist && g.rank() + 1 < g.nranks());
    if (g.trace) {
        g.rec("pro", {{"L", (long long)g.levelIndex(F)}, {"z1", z1}, {"z2", z2}, {"zlo", zlo}, {"zhi", zhi}});
        return;
    }
    // rows > 512 points (column blocks): the corrected edge columns go through a workspace, one per
    // stream (the boundary planes' launch runs beside the interior's)
    const int64_t wsn = gs_jacobi_sweep2_prolong_ws_elems(&g.stencilAbi, &sub, (int)g.mode);
    // (allocated once, at grid creation, for the largest plane range upLeg requests: never reallocated —
    // a hipFree / hipMalloc here would synchronise the device inside the overlapped sequence)
    DeviceBuf& wb = F.proWs[s == g.stream() ? 0 : 1];
    if (wsn > wb.size()) throw Error("gs_jacobi_sweep2_prolong: workspace not sized at grid creation");
    double* ws = wsn > 0 ? wb.get(wsn) : nullptr;
    check(gs_jacobi_sweep2_prolong_ws(&g.stencilAbi, &sub, g.kmode(), g.omega, g.gamma, F.v.data() + off,
                                      C.v.data(), nullptr, &C.geom, F.vAlt.data() + off, F.f.data() + off,
                                      g.wOf(F) ? g.wOf(F) + off : nullptr, zlo, zhi, ws, wsn, s),
          "gs_jacobi_sweep2_prolong");
}

} // namespace

// Workspace elements of the largest plane range upLeg's fused prolongation pair requests on level l
// (the whole level, or the boundary / interior ranges of the overlapped Z-slab sequence).
int64_t proWsElems(const HipGridData& g, std::size_t l)
{
    const gs_level& G = g.getLevel(l).geom;
    const int64_t nz = G.nz, zt = nz % 2 == 0 ? nz - 1 : nz - 2;
    const int64_t ranges[4][2] = {{1, nz}, {1, 2}, {zt, nz}, {3, zt - 1}};
    int64_t need = 0;
    for (const auto& r : ranges) {
        if (r[1] < r[0] || r[0] < 1) continue;
        gs_level sub = G;
        sub.nz = r[1] - r[0] + 1;
        sub.z0 += r[0] - 1;
        need = std::max(need, gs_jacobi_sweep2_prolong_ws_elems(&g.stencilAbi, &sub, (int)g.mode));
    }
    return need;
}

namespace {

bool transitionLevel(HipGridData& g, std::size_t l)
{
    return l > 0 && g.nranks() > 1 && !g.getLevel(l).distributed && g.getLevel(l - 1).distributed;
}

// fine level l -> coarse level l+1 (one or two coarse outputs), then ghost refresh / gather
void restrictTo(HipGridData& g, const DeviceField& src, std::size_t l, DeviceField& a, DeviceField* b,
                bool needGhosts)
{
    auto& F = g.getLevel(l);
    auto& C = g.getLevel(l + 1);
    const hipStream_t s = g.stream();
    int64_t off = 0;
    const gs_level cg = g.ownedGeom(C, &off);
    if (g.trace) {
        if (cg.nz > 0)
            g.rec("restrict", {{"L", (long long)l}, {"c1", cg.z0 + 1}, {"c2", cg.z0 + cg.nz}, {"two", b != nullptr}},
                  (std::string(HipGridData::fieldName(F, src)) + ">" + HipGridData::fieldName(C, a) +
                   (b ? std::string(",") + HipGridData::fieldName(C, *b) : std::string())).c_str());
    } else if (cg.nz > 0)
        check(gs_restrict2(src.data(), &F.geom, a.data() + off, b ? b->data() + off : nullptr, &cg, s), "gs_restrict");
    if (transitionLevel(g, l + 1)) {
        g.gather(C, a);
        if (b) g.gather(C, *b);
    } else if (needGhosts) {
        g.halo(C, a, s);
        if (b) g.halo(C, *b, s, g.vDepth(C)); // b is the coarse iterate (FAS)
    }
}

} // namespace

// The overlapped exchange of a Z-slab sweep: the boundary planes run on their own stream (forked
// from the compute stream), the exchange on the comm stream after them, and the interior planes on
// the compute stream concurrently with both; the compute stream waits for the exchange (join,
// recorded after it, waited on after the interior launch) before the next sweep. The boundary and
// interior launches write disjoint planes of vAlt and only read v. Nothing to order in trace mode.
hipStream_t HipSolver::forkBoundary(HipGridData& grid)
{
    if (grid.trace) return grid.stream();
    check((int)hipEventRecord(grid.evA_, grid.stream()), "hipEventRecord");
    check((int)hipStreamWaitEvent(grid.bndStream_.s, grid.evA_, 0), "hipStreamWaitEvent");
    return grid.bndStream_.s;
}

void HipSolver::forkComm(HipGridData& grid)
{
    if (grid.trace) return;
    check((int)hipEventRecord(grid.evC_, grid.bndStream_.s), "hipEventRecord");
    check((int)hipStreamWaitEvent(grid.commStream(), grid.evC_, 0), "hipStreamWaitEvent");
}

void HipSolver::joinComm(HipGridData& grid, bool wait)
{
    if (grid.trace) return;
    if (!wait) check((int)hipEventRecord(grid.evB_, grid.commStream()), "hipEventRecord");
    else check((int)hipStreamWaitEvent(grid.stream(), grid.evB_, 0), "hipStreamWaitEvent");
}

// the pipelined sequence's pending exchange settled on the host (its kernels are on the comm stream),
// then the event the next boundary planes and the final join wait on
void HipSolver::settleExchange(HipGridData& grid)
{
    grid.haloSettle();
    if (!grid.trace) check((int)hipEventRecord(grid.evB_, grid.commStream()), "hipEventRecord");
}

bool HipSolver::speculationEnabled(const HipGridData& grid)
{
    return grid.sw.speculation && grid.preSmoothing > 0 && grid.numLevels() > 1;
}

// src/cpu/CpuSolver.cpp:12-43. Every norm the loop reads (the initial one and each V-cycle's closing
// one) is the residual of the current level-0 iterate, which the next cycle's first pre-smoothing
// sweep computes anyway: that sweep runs speculatively into vAlt and reports the norm; if the loop
// stops there, vAlt is dropped and v is the final iterate, exactly as in the reference.
void HipSolver::solve(HipGridData& grid)
{
    const bool print = grid.printProgress && grid.rank() == 0;
    const bool spec = speculationEnabled(grid);
    int pending = 0;
    const double initialResidual = spec ? speculativeSweep(grid, &pending) : compResidual(grid, 0, false, true);
    if (history) history->push_back(initialResidual);
    if (print) std::cout << "Inital residual: " << initialResidual << '\n';
    if (print) Timer::start();
    auto onNorm = [&](std::size_t i, double res) {
        if (history) history->push_back(res);
        if (print) {
            std::cout << "iter: " << i << " residual: " << res << ' ';
            Timer::stop(); // "Took Nms": from the previous norm to this one (the cycles overlap)
            Timer::start();
        }
        return res <= initialResidual / (1.0 / grid.tol);
    };
    // The closing norm of the LAST cycle decides nothing (the loop ends at maxiter either way): when nobody
    // reads it — no progress print, no history, no per-level clock; NewtonSolver::findError's inner solves — that
    // cycle ends with its up-leg and the norm's pass (a whole level-0 pair at 512^3) is not run
    // (rank-uniform: every rank must run the same exchanges and collectives, so the decision rests on the
    // grid's printProgress, not on `print`, which only rank 0 has, and on clock.on, which a distributed grid
    // agrees across ranks at creation)
    const bool lastNormDead = !grid.printProgress && history == nullptr && !grid.clock.on;
    if (spec) {
        runCycles(grid, &pending, grid.maxiter, onNorm, lastNormDead);
    } else {
        for (std::size_t i = 0; i < grid.maxiter; i++) {
            if (lastNormDead && i + 1 == grid.maxiter) {
                cycleDown(grid, nullptr);
                cycleUpNoNorm(grid);
                break;
            }
            if (onNorm(i, vcycle(grid))) break;
        }
    }
}

// level 0's up-leg without the closing norm (the last cycle of a solve whose final norm nobody reads)
void HipSolver::cycleUpNoNorm(HipGridData& grid)
{
    if (std::min(grid.coarseFrom, grid.numLevels() - 1) >= 1) upLeg(grid, 1);
    if (grid.trace) grid.rec("nonorm", {{"L", 0}});
}

// Global ||.|| from this rank's per-block partials: fixed-order sums per rank, then over ranks in
// rank order, so every rank (and every run) gets the same bits.
double HipSolver::finishNorm(HipGridData& grid, int64_t nparts, bool wait)
{
    const hipStream_t s = grid.stream();
    if (grid.trace) {
        grid.rec("norm", {{"allgather", grid.nranks() > 1 && grid.getLevel(0).distributed}});
        return wait ? grid.readNorm() : std::nan(""); // (!wait: readNormEnd reads it)
    }
    if (grid.nranks() > 1 && grid.getLevel(0).distributed) {
        check(gs_sumsq_finish(grid.partials(), nparts, grid.dNorm(), 1, s), "gs_sumsq_finish");
        grid.comm()->allgather1(grid.dNorm(), grid.dRankSums(), s);
        check(gs_sumsq_finish(grid.dRankSums(), grid.nranks(), grid.hNormDev(), 0, s), "gs_sumsq_finish");
    } else {
        check(gs_sumsq_finish(grid.partials(), nparts, grid.hNormDev(), 0, s), "gs_sumsq_finish");
    }
    if (wait) return grid.readNorm();
    grid.readNormBegin();
    return std::nan("");
}

// compResidual (src/cpu/CpuSolver.cpp:45-83): r is written only when a restriction consumes it,
// the norm only when a caller reads it (level 0).
double HipSolver::compResidual(HipGridData& grid, std::size_t l, bool storeR, bool norm)
{
    materialize(grid, l);
    auto& L = grid.getLevel(l);
    const hipStream_t s = grid.stream();
    if (grid.trace)
        grid.rec("residual", {{"L", (long long)l}, {"store", storeR}, {"norm", norm}});
    else
        check(gs_residual(&grid.stencilAbi, &L.geom, grid.kmode(), grid.gamma, L.v.data(), L.f.data(),
                          grid.wOf(L), storeR ? L.r.data() : nullptr,
                          norm ? grid.partials() : nullptr, s),
              "gs_residual");
    if (storeR) grid.halo(L, L.r, s);
    if (!norm) return 0.0;
    return finishNorm(grid, gs_residual_num_partials(&grid.stencilAbi, &L.geom));
}

// Whether level l's first post-smoothing pair can take the prolongation from level l+1 (rank-uniform:
// the pair's ghost exchange is collective). A Z-slab level needs every slab to start on an even global
// plane (the kernel's plane parities) and, under a Z-slab coarse level, each rank's coarse planes over
// its fine ones with two coarse ghost planes (the bottom ghost fine plane interpolates from coarse
// plane -1); a replicated coarse level holds every plane.
static bool proSlabOk(HipGridData& grid, std::size_t l)
{
    auto& F = grid.getLevel(l);
    auto& C = grid.getLevel(l + 1);
    if (!(F.distributed && grid.nranks() > 1)) return true;
    for (int q = 0; q < grid.nranks(); q++) {
        if ((F.ranksLo[q] - 1) % 2 != 0) return false;
        if (C.distributed && 2 * (C.ranksLo[q] - 1) != F.ranksLo[q] - 1) return false;
    }
    return !C.distributed || grid.vDepth(C) == 2;
}

// NEWTON's fused prolongation pair keeps part of its state in LDS and recomputes exp(newtonV) for
// its second sweep: on 512^3 it saves 0.14 ms per V-cycle against gs_prolong_add + the plain pair, on
// 256^3 / 128^3 it cost 0.065 / 0.05 ms more (profiles/r01l_summary.md). Since r04 levels of at most
// two 256-point y-blocks launch a two-x-wave instance (74 KB of LDS, two blocks per CU), which wins on
// 512^3's level 1 and 256^3's level 0 too (Newton iteration 36.5-36.6 against 36.7-36.75 ms at 512^3,
// 6.32-6.36 against 6.58-6.62 ms at 256^3: profiles/r04/r04e_newton_ab_swizzle_rrreverse.txt,
// r04f_newton_pro_threshold.txt),
// so NEWTON levels take it from GS_NEWTON_PRO_POINTS points per rank on (judged on the thinnest slab: rank-uniform).
// Since r06 the default is 2^21, so 512^3's 128^3 level fuses too: its two-x-wave GS_NEWTON_B prolongation pair
// (34.7 us) replaces gs_prolong_add (39 us) + the plain pair (22 us), one launch fewer per inner V-cycle; a Newton
// iteration's kernel time 29.09 vs 29.22 ms, wall 27.63-27.80 vs 27.69-27.84 ms (3 interleaved rounds,
// profiles/r06/r06p_newton_pro_points_ab.txt). LINEAR levels always do.
static bool proWorthIt(HipGridData& grid, std::size_t l)
{
    if (grid.mode != GridParams::NEWTON) return true;
    const int64_t minPoints = grid.sw.newtonProPoints;
    const auto& F = grid.getLevel(l);
    return (int64_t)F.levelDim[0] * (int64_t)F.levelDim[1] * F.minPlanes >= minPoints;
}

// k sweeps (src/cpu/CpuSolver.cpp:141-180). Each reads v and writes vAlt, then the two swap. Where
// the level allows, sweeps run in fused pairs (gs_jacobi_sweep2: one read of v and f, one write, for
// two sweeps), an odd one as a single sweep.
//
// On a Z-slab the outermost planes of each step (one per side for a sweep, two for a pair) run on the
// boundary stream, their ghost exchange follows on the comm stream, and the interior planes run on the
// compute stream beside both. The steps of one call are pipelined so that the compute stream never waits
// for an exchange: step k's interior reads only v's owned planes (k-1's interior, k-1's boundary
// planes), never its ghost planes, so it needs boundary k-1 but not exchange k-1. Only the boundary
// planes of step k wait for exchange k-1 (the ghosts they read) and for interior k-1 (whose input planes
// they overwrite); exchange k then hides under interior k+1 instead of sitting between two interiors.
// The last exchange is joined into the compute stream before returning. Writes never meet a read of the
// same planes: interior k writes the buffer exchange k-2 sent from (its boundary planes only) and that
// boundary k-1 read planes 3-4 of before it (event), boundary k writes planes exchange k-2 sent (comm is
// in order, boundary k waits exchange k-1). The interior launch is enqueued before the exchange is issued:
// RCCL's non-blocking group is settled on the host (gs_comm.cpp), and the GPU must not wait on that host
// round-trip between the boundary planes and the interior.
void HipSolver::jacobi(HipGridData& grid, std::size_t l, std::size_t sweeps)
{
    auto& L = grid.getLevel(l);
    const hipStream_t s = grid.stream();
    const bool dist = L.distributed && grid.nranks() > 1;
    const int64_t nz = L.geom.nz;
    const int depth = grid.vDepth(L);
    int step = 0; // overlapped steps issued in this call
    while (sweeps > 0) {
        const bool pair = L.fusedPairs && sweeps >= 2;
        const int64_t b = pair ? 2 : depth; // outermost planes whose ghost copies the neighbours need
        auto run = [&](int64_t z1, int64_t z2, hipStream_t st) {
            if (pair) pairPlanes(grid, L, z1, z2, st);
            else sweepPlanes(grid, L, z1, z2, st);
        };
        if (!dist) {
            run(1, nz, s);
        } else if (grid.overlapHalo && nz >= 2 * b + 1) {
            hipStream_t bs = s;
            // interior k reads boundary k-1's planes (boundary k's event slot is recorded below, k-1's still
            // holds) and interior k-1's, but no ghost plane: it may go before exchange k-1 has settled. When
            // that exchange is still being settled on the host (RCCL's non-blocking group), interior k is
            // enqueued first, so the GPU never idles behind the host; otherwise boundary k goes first, so its
            // exchange starts as early as possible (GS_HALO_ORDER forces either order)
            const bool interiorFirst = step > 0 && !grid.haloReady();
            if (!grid.trace) {
                bs = grid.bndStream_.s;
                check((int)hipEventRecord(grid.evA_, s), "hipEventRecord"); // after interior k-1
            }
            auto interior = [&] {
                if (!grid.trace && step > 0)
                    check((int)hipStreamWaitEvent(s, grid.evBnd_[(step - 1) & 1], 0), "hipStreamWaitEvent");
                run(b + 1, nz - b, s);
            };
            if (interiorFirst) interior();
            if (step > 0) settleExchange(grid); // exchange k-1's kernels on the comm stream, then evB
            if (!grid.trace) {
                // boundary k after interior k-1 (whose input planes it overwrites) and after exchange k-1
                // (the ghost planes it reads; on the comm stream, after every earlier exchange)
                check((int)hipStreamWaitEvent(bs, grid.evA_, 0), "hipStreamWaitEvent");
                if (step > 0) check((int)hipStreamWaitEvent(bs, grid.evB_, 0), "hipStreamWaitEvent");
            }
            run(1, b, bs);
            run(nz - b + 1, nz, bs);
            if (!grid.trace) {
                hipEvent_t bnd = grid.evBnd_[step & 1];
                check((int)hipEventRecord(bnd, bs), "hipEventRecord");
                check((int)hipStreamWaitEvent(grid.commStream(), bnd, 0), "hipStreamWaitEvent");
            }
            if (!interiorFirst) interior();
            grid.haloIssue(L, L.vAlt, grid.commStream(), depth); // settled at the next step or below
            step++;
        } else {
            if (step > 0) {
                settleExchange(grid);
                joinComm(grid, true); // an earlier overlapped step's exchange
            }
            step = 0;
            run(1, nz, s);
            grid.halo(L, L.vAlt, s, depth);
        }
        L.v.swap(L.vAlt);
        if (grid.trace) grid.rec("swap", {{"L", (long long)l}});
        L.vZero = false;
        sweeps -= pair ? 2 : 1;
    }
    if (step > 0) {
        // the last exchange (and through it the last boundary planes) before anything else on the level
        settleExchange(grid);
        joinComm(grid, true);
        if (!grid.trace) check((int)hipStreamWaitEvent(s, grid.evBnd_[(step - 1) & 1], 0), "hipStreamWaitEvent");
    }
}

// v = 0 made real (the zero-iterate sweeps had no chance to replace it)
void HipSolver::materialize(HipGridData& grid, std::size_t l)
{
    auto& L = grid.getLevel(l);
    if (!L.vZero) return;
    if (grid.trace) grid.rec("zero", {{"L", (long long)l}}, "v");
    L.v.zero(grid.stream());
    L.vZero = false;
}

// CpuSolver.cpp:92-135 below level `from` in one launch (gs_coarse_cycle): the caller has set
// f^from (and, FAS, restV / v); on return every level from..nl-1 holds its post-smoothed iterate.
void HipSolver::coarseCycle(HipGridData& grid, std::size_t from)
{
    const std::size_t nl = grid.numLevels();
    gs_coarse_level lv[16] = {};
    const int n = (int)(nl - from);
    if (n < 1 || n > 16) throw Error("coarseCycle: bad level range");
    for (int j = 0; j < n; j++) {
        auto& L = grid.getLevel(from + j);
        lv[j] = gs_coarse_level{L.v.data(), L.vAlt.data(), L.f.data(), L.r ? L.r.data() : nullptr,
                                L.restV ? L.restV.data() : nullptr, const_cast<double*>(grid.wOf(L)),
                                L.geom, j == 0 ? (L.vZero ? 1 : 0) : (grid.mode != GridParams::NONLINEAR ? 1 : 0)};
    }
    if (grid.trace)
        grid.rec("coarse", {{"from", (long long)from}, {"vzero", lv[0].v_zero}});
    else
        check(gs_coarse_cycle(&grid.stencilAbi, lv, n, grid.kmode(), grid.omega, grid.gamma, (int)grid.preSmoothing,
                              (int)grid.postSmoothing, grid.stream()),
              "gs_coarse_cycle");
    const bool odd = ((grid.preSmoothing + grid.postSmoothing) & 1) != 0; // every level swept pre+post times
    for (int j = 0; j < n; j++) {
        auto& L = grid.getLevel(from + j);
        if (odd) {
            L.v.swap(L.vAlt);
            if (grid.trace) grid.rec("swap", {{"L", (long long)(from + j)}});
        }
        L.vZero = false;
    }
}

// The first pre-smoothing step of the next cycle, run into vAlt (v untouched) with the norm of the
// residual of v: a fused pair when level 0 smooths in pairs and pre-smoothing has two sweeps, else
// one sweep. *sweeps = how many sweeps vAlt holds.
double HipSolver::speculativeSweep(HipGridData& grid, int* sweeps, bool wait)
{
    auto& L = grid.getLevel(0);
    const hipStream_t s = grid.stream();
    const int64_t nz = L.geom.nz;
    double* P = grid.partials();
    int64_t n = 0;
    const bool pair = L.fusedPairs && grid.preSmoothing >= 2;
    const int depth = grid.vDepth(L);
    const int64_t b = pair ? 2 : depth;
    auto run = [&](int64_t z1, int64_t z2, hipStream_t st) {
        n += pair ? pairPlanes(grid, L, z1, z2, st, P + n) : sweepPlanes(grid, L, z1, z2, st, P + n);
    };
    if (!(L.distributed && grid.nranks() > 1)) {
        run(1, nz, s);
    } else if (grid.overlapHalo && nz >= 2 * b + 1) {
        const hipStream_t bs = forkBoundary(grid);
        run(1, b, bs);
        run(nz - b + 1, nz, bs);
        forkComm(grid);
        run(b + 1, nz - b, s); // interior enqueued before the RCCL group is issued and settled
        grid.halo(L, L.vAlt, grid.commStream(), depth);
        joinComm(grid, false);
        joinComm(grid, true);
    } else {
        run(1, nz, s);
        grid.halo(L, L.vAlt, s, depth);
    }
    if (sweeps) *sweeps = pair ? 2 : 1;
    grid.clock.mark(s, 0, false); // closes the caller's segment before the norm's host sync
    return finishNorm(grid, n, wait);
}

void HipSolver::restrict(HipGridData& grid, const DeviceField& src, std::size_t srcLevel, DeviceField& dst)
{
    restrictTo(grid, src, srcLevel, dst, nullptr, true);
}

double HipSolver::vcycle(HipGridData& grid) { return vcycleSpeculative(grid, nullptr); }

// The up-leg of level i-1 from level i (CpuSolver.cpp:121-135): v^(i-1) += P v^i, post-smoothing.
void HipSolver::upLeg(HipGridData& grid, std::size_t i)
{
    const hipStream_t s = grid.stream();
    auto& C = grid.getLevel(i);
    auto& F = grid.getLevel(i - 1);
    grid.clock.mark(s, (int)(i - 1), true);
    materialize(grid, i); // only if the level had no sweep at all
    // (the tiled step fuses the prolongation with a pair: the GS_NO_FUSED_SWEEPS / GS_NO_FUSED_PROLONG
    // alternatives take the general path below)
    if (i - 1 >= 1 && F.tiled && !C.distributed && grid.postSmoothing >= 2 && grid.sw.fusedSweeps &&
        grid.sw.fusedProlong) {
        // a small level: prolongation, correction and the first two post-smoothing sweeps in one launch
        materialize(grid, i - 1);
        if (grid.trace)
            grid.rec("tiledpro", {{"L", (long long)(i - 1)}});
        else
            check(gs_prolong_smooth2_tiled(&grid.stencilAbi, &F.geom, grid.kmode(), grid.omega, grid.gamma,
                                           F.v.data(), C.v.data(), &C.geom, F.vAlt.data(), F.f.data(),
                                           grid.wOf(F), s),
                  "gs_prolong_smooth2_tiled");
        F.v.swap(F.vAlt);
        if (grid.trace) grid.rec("swap", {{"L", (long long)(i - 1)}});
        F.vZero = false;
        jacobi(grid, i - 1, grid.postSmoothing - 2);
        grid.clock.mark(s, (int)(i - 1), false);
        return;
    }
    if (grid.sw.fusedProlong && F.fusedPairs && grid.postSmoothing >= 2 && proWorthIt(grid, i - 1) && proSlabOk(grid, i - 1) &&
        gs_jacobi_sweep2_prolong_supported(&grid.stencilAbi, &F.geom, (int)grid.mode)) {
        // the first two post-smoothing sweeps of v^h + P v^2h in one pass (the corrected
        // iterate is never stored), then the remaining ones. On a Z-slab each rank corrects its
        // ghost planes itself, from the coarse planes under them, and the pair's outermost planes
        // go first so that their exchange overlaps the interior (as in jacobi())
        materialize(grid, i - 1);
        const int64_t nz = F.geom.nz;
        if (!(F.distributed && grid.nranks() > 1)) {
            proPlanes(grid, F, C, 1, nz, s);
        } else if (grid.overlapHalo && nz >= 5) {
            const int64_t zt = nz % 2 == 0 ? nz - 1 : nz - 2; // odd start: 2 or 3 top planes
            const hipStream_t bs = forkBoundary(grid);
            proPlanes(grid, F, C, 1, 2, bs);
            proPlanes(grid, F, C, zt, nz, bs);
            forkComm(grid);
            proPlanes(grid, F, C, 3, zt - 1, s); // interior first (see jacobi())
            grid.halo(F, F.vAlt, grid.commStream(), grid.vDepth(F));
            joinComm(grid, false);
            joinComm(grid, true);
        } else {
            proPlanes(grid, F, C, 1, nz, s);
            grid.halo(F, F.vAlt, s, grid.vDepth(F));
        }
        F.v.swap(F.vAlt);
        if (grid.trace) grid.rec("swap", {{"L", (long long)(i - 1)}});
        F.vZero = false;
        jacobi(grid, i - 1, grid.postSmoothing - 2);
        grid.clock.mark(s, (int)(i - 1), false);
        return;
    }
    // v^h += P (v^2h [- restV^2h])   (CpuSolver.cpp:121-132, interpolate + v += e fused)
    if (grid.trace)
        grid.rec("prolongadd", {{"L", (long long)(i - 1)}, {"sub", grid.mode == GridParams::NONLINEAR}});
    else
        check(gs_prolong_add(C.v.data(), grid.mode == GridParams::NONLINEAR ? C.restV.data() : nullptr, &C.geom,
                             F.v.data(), &F.geom, s),
              "gs_prolong_add");
    grid.halo(F, F.v, s, grid.vDepth(F));
    jacobi(grid, i - 1, grid.postSmoothing);
    grid.clock.mark(s, (int)(i - 1), false);
}

// src/cpu/CpuSolver.cpp:85-139, in two halves (see gs_grid.hpp)
void HipSolver::cycleDown(HipGridData& grid, int* pending)
{
    const std::size_t nl = grid.numLevels();
    const hipStream_t s = grid.stream();
    // levels lc.. run as one gs_coarse_cycle launch (lc == nl: none); the host loops descend to lc
    const std::size_t lc = grid.coarseFrom, last = std::min(lc, nl - 1);
    for (std::size_t i = 0; i < last; i++) {
        grid.clock.mark(s, (int)i, true);
        std::size_t pre = grid.preSmoothing;
        if (i == 0 && pending && *pending > 0 && pre >= (std::size_t)*pending) {
            grid.getLevel(0).v.swap(grid.getLevel(0).vAlt); // adopt the speculative first sweep(s)
            grid.getLevel(0).vZero = false;
            if (grid.trace) grid.rec("swap", {{"L", 0}});
            pre -= (std::size_t)*pending;
            *pending = 0;
        }
        auto& L = grid.getLevel(i);
        auto& C = grid.getLevel(i + 1);
        // (the tiled step fuses a pair, the residual and the restriction and leaves v^2h = 0 as a flag: the
        // GS_NO_FUSED_SWEEPS / GS_NO_FUSED_RR / GS_NO_ZERO_GUESS alternatives take the general path below)
        if (i >= 1 && pre == 2 && L.tiled && !C.distributed && grid.sw.fusedSweeps && grid.sw.fusedRR &&
            grid.sw.zeroGuess) {
            // a small level: the pre-smoothing pair, residual and restriction in one tiled launch
            if (grid.trace)
                grid.rec("tiledpre", {{"L", (long long)i}, {"vzero", L.vZero}});
            else
                check(gs_smooth2_restrict_tiled(&grid.stencilAbi, &L.geom, grid.kmode(), grid.omega, grid.gamma,
                                                L.vZero ? nullptr : L.v.data(), L.vAlt.data(), L.f.data(),
                                                grid.wOf(L), C.f.data(), &C.geom, s),
                      "gs_smooth2_restrict_tiled");
            L.v.swap(L.vAlt);
            if (grid.trace) grid.rec("swap", {{"L", (long long)i}});
            L.vZero = false;
            C.vZero = true; // LINEAR / NEWTON: v^2h = 0 (CpuSolver.cpp:100-101), not stored
            grid.clock.mark(s, (int)i, false);
            continue;
        }
        jacobi(grid, i, pre);
        // f^2h = R (f^h - A v^h) in one pass: the fine residual is never stored
        bool fused = false;
        if (grid.sw.fusedRR) {
            materialize(grid, i);
            const double* w = grid.wOf(L);
            if (!(L.distributed && grid.nranks() > 1)) {
                if (grid.trace)
                    grid.rec("resrestrict", {{"L", (long long)i}, {"c1", 1}, {"c2", C.geom.nz}, {"zhi", 0}});
                else
                    check(gs_residual_restrict(&grid.stencilAbi, &L.geom, grid.kmode(), grid.gamma, L.v.data(),
                                               L.f.data(), w, C.f.data(), nullptr, &C.geom, s),
                          "gs_residual_restrict");
                fused = true;
            } else {
                // Z-slab: this rank's coarse planes from its fine slab, whose top ghost planes are current
                // (v after the sweep's exchange, f / newtonV after theirs); then the coarse ghosts / gather
                // every rank must take the same branch (the ghost exchanges are collective): the slab
                // kernel needs each rank's coarse planes over its even fine planes
                bool slabOk = true;
                for (int q = 0; q < grid.nranks(); q++)
                    if (C.ranksHi[q] >= C.ranksLo[q]) slabOk = slabOk && 2 * (C.ranksLo[q] - 1) == L.ranksLo[q] - 1;
                int64_t off = 0;
                const gs_level cg = grid.ownedGeom(C, &off);
                const int zhi = grid.rank() + 1 < grid.nranks();
                // (the residual on the top ghost plane reads v two planes deep)
                slabOk = slabOk && grid.vDepth(L) == 2 &&
                         gs_residual_restrict_slab_supported(&grid.stencilAbi, &L.geom) != 0;
                if (slabOk) {
                    if (cg.nz > 0 && grid.trace)
                        grid.rec("resrestrict", {{"L", (long long)i}, {"c1", cg.z0 + 1}, {"c2", cg.z0 + cg.nz}, {"zhi", zhi}});
                    else if (cg.nz > 0)
                        check(gs_residual_restrict_slab(&grid.stencilAbi, &L.geom, grid.kmode(), grid.gamma,
                                                        L.v.data(), L.f.data(), w, C.f.data() + off, nullptr, &cg,
                                                        zhi, s),
                              "gs_residual_restrict_slab");
                    if (transitionLevel(grid, i + 1)) grid.gather(C, C.f);
                    else grid.halo(C, C.f, s);
                    fused = true;
                }
            }
        }
        if (!fused) {
            compResidual(grid, i, true, false);
            restrictTo(grid, L.r, i, C.f, nullptr, true); // f^2h = R r^h (ghosts: the fused pair reads them)
        }
        if (grid.mode != GridParams::NONLINEAR) {
            // v^2h = 0 (CpuSolver.cpp:114-116): not stored; the first sweep on the level reads no v
            if (!grid.sw.zeroGuess) {
                if (grid.trace) grid.rec("zero", {{"L", (long long)(i + 1)}}, "v");
                C.v.zero(s);
            } else {
                C.vZero = true;
            }
        } else {
            // FAS: restV = v^2h = R v^h, then f^2h += A^2h(restV)  (CpuSolver.cpp:104-113)
            restrictTo(grid, L.v, i, C.restV, &C.v, true);
            if (grid.trace)
                grid.rec("applyadd", {{"L", (long long)(i + 1)}});
            else
                check(gs_apply_op_add(&grid.stencilAbi, &C.geom, grid.gamma, C.restV.data(), C.f.data(), s),
                      "gs_apply_op_add");
            grid.halo(C, C.f, s);
        }
        grid.clock.mark(s, (int)i, false);
    }
    grid.clock.mark(s, (int)std::min(lc, nl - 1), true);
    if (lc < nl) coarseCycle(grid, lc);
    else jacobi(grid, nl - 1, grid.preSmoothing + grid.postSmoothing); // coarsest "solve"
    grid.clock.mark(s, (int)std::min(lc, nl - 1), false);
    for (std::size_t i = last; i > 1; i--) upLeg(grid, i);
}

double HipSolver::cycleUp0(HipGridData& grid, int* pending, bool wait)
{
    const std::size_t nl = grid.numLevels();
    const hipStream_t s = grid.stream();
    if (std::min(grid.coarseFrom, nl - 1) >= 1) upLeg(grid, 1);
    // the closing norm: the next cycle's first pre-smoothing step (speculative) or a residual pass
    grid.clock.mark(s, 0, true);
    double res;
    if (pending && speculationEnabled(grid)) {
        res = speculativeSweep(grid, pending, wait); // closes the segment before its host sync
    } else {
        res = compResidual(grid, 0, false, true);
        grid.clock.mark(s, 0, false); // after the norm's host sync: over-counts by the sync latency
    }
    return res;
}

double HipSolver::vcycleSpeculative(HipGridData& grid, int* pending)
{
    const auto tWall = std::chrono::steady_clock::now();
    cycleDown(grid, pending);
    const double res = cycleUp0(grid, pending, true);
    if (grid.clock.on) {
        grid.clock.collect();
        grid.clock.cycles++;
        grid.clock.wallMs += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tWall).count();
    }
    return res;
}

// Overlapping cycle i+1's cycleDown with the wait for cycle i's norm is exact only if that work
// leaves level 0's iterate alone: every pre-smoothing sweep is the speculative step's (pre ==
// pending), level 0 is not part of the coarse-cycle launch, and no per-level clock is running.
bool HipSolver::pipelinable(const HipGridData& grid, int pending)
{
    return grid.sw.pipeline && !grid.clock.on && speculationEnabled(grid) && pending > 0 &&
           (std::size_t)pending == grid.preSmoothing && std::min(grid.coarseFrom, grid.numLevels() - 1) >= 1;
}

std::size_t HipSolver::runCycles(HipGridData& grid, int* pending, std::size_t maxCycles,
                                 const std::function<bool(std::size_t, double)>& onNorm, bool lastNormDead)
{
    // (cycle-invariant: every closing speculative step leaves the same number of sweeps pending)
    const bool pipe = pipelinable(grid, *pending);
    bool downDone = false; // this cycle's cycleDown was enqueued during the previous cycle's wait
    for (std::size_t i = 0; i < maxCycles; i++) {
        if (lastNormDead && i + 1 == maxCycles) {
            // the last cycle's closing norm decides nothing and nobody reads it: no speculative pass
            if (!downDone) cycleDown(grid, pending);
            cycleUpNoNorm(grid);
            *pending = 0;
            return maxCycles;
        }
        if (!pipe) {
            if (onNorm(i, vcycleSpeculative(grid, pending))) return i + 1;
            continue;
        }
        if (!downDone) cycleDown(grid, pending);
        cycleUp0(grid, pending, false); // cycle i's closing norm in flight; *pending = its sweeps
        const int next = *pending;
        const bool ahead = i + 1 < maxCycles;
        if (ahead) cycleDown(grid, pending); // adopts the speculative sweeps: *pending = 0
        const double res = grid.readNormEnd();
        if (onNorm(i, res)) {
            if (ahead) { // undo the adoption: level 0 holds cycle i's iterate, vAlt the speculation
                auto& L0 = grid.getLevel(0);
                L0.v.swap(L0.vAlt);
                if (grid.trace) grid.rec("swap", {{"L", 0}});
                *pending = next;
            }
            return i + 1;
        }
        downDone = ahead;
    }
    return maxCycles;
}

void NewtonSolver::solve(HipGridData& grid)
{
    auto& L0 = grid.getLevel(0);
    const hipStream_t s = grid.stream();
    // the reference prints unconditionally (NewtonSolver.cpp:16,27); printProgress defaults to true,
    // so GpuSolve-hip does too, and library callers silence it without touching std::cout
    const bool print = grid.printProgress && grid.rank() == 0;
    if (grid.trace)
        grid.rec("copy", {{"L", 0}}, "f>newtonF");
    else
        check(gs_copy(grid.newtonF.data(), L0.f.data(), L0.f.span(), s), "gs_copy");
    const double initialResidual = compF(grid);
    // fields may have been set since the last solve: the first findError restricts level 1 and forms level 0's factor
    // itself, and skips the restrictions of a zero newtonV only if EVERY rank still has it (a rank that handed its
    // newtonV pointer out would restrict, and restrictions exchange ghost planes on distributed levels)
    grid.newtonR1_ = false;
    grid.bfacFresh_ = 0;
    grid.newtonVZero_ = grid.allRanks(grid.newtonVZero_);
    if (history) history->push_back(initialResidual);
    if (print) std::cout << "Inital newton residual: " << initialResidual << '\n';

    for (std::size_t i = 0; i < grid.maxiter; i++) {
        if (print) Timer::start();
        // The reference recomputes compF here (NewtonSolver.cpp:21); f^0 already holds exactly that
        // value from the previous compF and nothing wrote it since, so the pass is skipped.
        // v = 0 (NewtonSolver.cpp:22), not stored: the inner solve's first (speculative) sweep is a
        // zero-iterate kernel that reads no v; anything else that reads v materializes it first
        L0.vZero = true;
        const double res = findError(grid) ? compFUpdate(grid) : compF(grid);
        if (history) history->push_back(res);
        if (print) {
            std::cout << "newton iter: " << i << " residual: " << res << ' ';
            Timer::stop();
        }
        if (res <= initialResidual / (1.0 / grid.tol)) return;
    }
}

// f^0 = newtonF - N(newtonV^0), returns ||f^0||  (NewtonSolver.cpp:48-81)
double NewtonSolver::compF(HipGridData& grid)
{
    auto& L0 = grid.getLevel(0);
    if (grid.trace)
        grid.rec("newtonF", {{"L", 0}});
    else
        check(gs_newton_F(&grid.stencilAbi, &L0.geom, grid.gamma, L0.newtonV.data(), grid.newtonF.data(),
                          L0.f.data(), grid.partials(), grid.stream()),
              "gs_newton_F");
    grid.halo(L0, L0.f, grid.stream());
    return HipSolver::finishNorm(grid, gs_residual_num_partials(&grid.stencilAbi, &L0.geom));
}

// newtonV += v and the compF after it as one pass (gs_newton_F_update) on a level this rank holds whole:
// the sum goes to level 0's vAlt — zero outside the interior like newtonV + v, and dead once the inner
// solve has returned (its pending speculative sweep is dropped; the next inner solve starts from the
// zero iterate) — which then becomes newtonV. Bit-identical to gs_axpy + gs_newton_F.
// On a Z-slab rank the pass reads w and e on the ghost planes 0 and nz+1 (both current: newtonV's from the
// previous update, v's from the inner solve's last exchange) but stores w' only on the owned planes, so
// the new newtonV's ghost planes are formed afterwards as k_axpy would leave them (newtonV + 1.0 v, two
// planes: a copy and an axpy each) — no exchange, bit-identical to the whole-array gs_axpy of the
// two-pass path.
bool NewtonSolver::fusedUpdate(const HipGridData& grid)
{
    const auto& L0 = grid.getLevel(0);
    return grid.sw.newtonFusedUpdate && gs_newton_F_update_supported(&grid.stencilAbi, &L0.geom) != 0;
}

double NewtonSolver::compFUpdate(HipGridData& grid)
{
    auto& L0 = grid.getLevel(0);
    // single GPU: the next findError's restriction of newtonV onto level 1 (NewtonSolver.cpp:88-92) comes out of
    // the same pass (gs_newton_F_update_restrict), so findError skips that 1.1 GB re-read at 512^3
    const bool r1 = grid.numLevels() >= 3 && !(L0.distributed && grid.nranks() > 1) &&
                    (grid.trace || grid.getLevel(1).newtonVNext.data() != nullptr) &&
                    gs_newton_F_update_restrict_supported(&grid.stencilAbi, &L0.geom, &grid.getLevel(1).geom) != 0;
    // the same pass also writes the next inner solve's GS_NEWTON_B factor of level 0 (from the exp(w') compF
    // evaluates anyway): findError then skips that level's gs_newton_bfac pass
    const bool bf = r1 && grid.sw.newtonB && grid.sw.newtonBFused;
    if (grid.trace)
        grid.rec("newtonFupdate", {{"L", 0}, {"restrict", r1}, {"bfac", bf}});
    else if (r1)
        check(gs_newton_F_update_restrict_bfac(&grid.stencilAbi, &L0.geom, grid.gamma, L0.newtonV.data(), L0.v.data(),
                                               grid.newtonF.data(), L0.vAlt.data(), L0.f.data(), grid.partials(),
                                               grid.getLevel(1).newtonVNext.data(), &grid.getLevel(1).geom,
                                               bf ? L0.bfac.data() : nullptr, grid.stream()),
              "gs_newton_F_update_restrict");
    else
        check(gs_newton_F_update(&grid.stencilAbi, &L0.geom, grid.gamma, L0.newtonV.data(), L0.v.data(),
                                 grid.newtonF.data(), L0.vAlt.data(), L0.f.data(), grid.partials(), grid.stream()),
              "gs_newton_F_update");
    grid.newtonR1_ = r1;
    grid.bfacFresh_ = bf ? 1u : 0u;
    grid.newtonVZero_ = false;
    if (L0.distributed && grid.nranks() > 1) {
        // the ghost planes of w' = newtonV + v (see fusedUpdate)
        const int64_t ldz = L0.v.ldz();
        for (const int64_t p : {(int64_t)0, L0.geom.nz + 1}) {
            if (grid.trace) {
                grid.rec("ghostsum", {{"L", 0}, {"plane", (long long)p}}, "vAlt=newtonV+v");
                continue;
            }
            check(gs_copy(L0.vAlt.data() + p * ldz, L0.newtonV.data() + p * ldz, ldz, grid.stream()), "gs_copy");
            check(gs_axpy(L0.vAlt.data() + p * ldz, L0.v.data() + p * ldz, 1.0, ldz, grid.stream()), "gs_axpy");
        }
    }
    L0.newtonV.swap(L0.vAlt);
    if (grid.trace) grid.rec("swapnewton", {{"L", 0}});
    grid.halo(L0, L0.f, grid.stream());
    return HipSolver::finishNorm(grid, gs_residual_num_partials(&grid.stencilAbi, &L0.geom));
}

// NewtonSolver.cpp:83-108
bool NewtonSolver::findError(HipGridData& grid)
{
    // newtonV is still the zero every level's field was created with (the first Newton iteration): its
    // restrictions are those zeros (nothing to compute) and every factor is B = gamma (1 + 0) exp(0) = gamma
    const bool zeroW = grid.newtonVZero_;
    for (std::size_t i = 1; !zeroW && i + 1 < grid.numLevels(); i++) {
        if (i == 1 && grid.newtonR1_) { // restricted by the last compFUpdate; level 0's newtonV unchanged since
            grid.getLevel(1).newtonV.swap(grid.getLevel(1).newtonVNext);
            if (grid.trace) grid.rec("swapnewton", {{"L", 1}});
            grid.newtonR1_ = false;
            continue;
        }
        HipSolver::restrict(grid, grid.getLevel(i - 1).newtonV, i - 1, grid.getLevel(i).newtonV);
    }
    // GS_NEWTON_B: every level's factor B = gamma (1 + w) exp(w) of the newtonV the inner solve linearises at
    // (whole local arrays, ghost planes included: each level's newtonV ghosts are current here), so its ten
    // V-cycles evaluate no exp(newtonV) (include/gpusolve_hip.h)
    if (grid.sw.newtonB) {
        for (std::size_t i = 0; i < grid.numLevels(); i++) {
            auto& L = grid.getLevel(i);
            if (i < 32 && (grid.bfacFresh_ >> i) & 1u) continue; // written by the last compFUpdate pass
            if (grid.trace) grid.rec("bfac", {{"L", (long long)i}});
            else if (zeroW) // (planes -1 .. nz+2, as gs_newton_bfac covers)
                check(gs_fill(L.bfac.data() - L.bfac.ldz(), grid.gamma * (1 + 0.0) * std::exp(0.0),
                              L.bfac.ldz() * (L.geom.nz + 4), grid.stream()),
                      "gs_fill");
            else check(gs_newton_bfac(&L.geom, grid.gamma, L.newtonV.data(), L.bfac.data(), grid.stream()), "gs_newton_bfac");
        }
        grid.newtonB_ = true;
        grid.bconst_ = zeroW && grid.sw.newtonG; // B = gamma everywhere: GS_NEWTON_G
    }
    grid.bfacFresh_ = 0;

    const bool keepPrint = grid.printProgress;
    grid.printProgress = false;
    const std::size_t origIter = grid.maxiter;
    const double origTol = grid.tol;
    grid.maxiter = 10;
    grid.tol = 0.1;
    std::vector<double>* keep = HipSolver::history;
    HipSolver::history = nullptr;
    try {
        HipSolver::solve(grid);
    } catch (...) {
        grid.newtonB_ = grid.bconst_ = false;
        throw;
    }
    grid.newtonB_ = grid.bconst_ = false; // newtonV changes next (newtonV += v): the factors are stale from here on
    HipSolver::history = keep;
    grid.printProgress = keepPrint;
    grid.maxiter = origIter;
    grid.tol = origTol;

    if (fusedUpdate(grid)) return true; // compFUpdate adds v
    auto& L0 = grid.getLevel(0);
    // whole local array, ghost planes included: both operands' ghosts are current, so the sum's are
    if (grid.trace) grid.rec("axpy", {{"L", 0}}, "newtonV+=v");
    else check(gs_axpy(L0.newtonV.data(), L0.v.data(), 1.0, L0.v.span(), grid.stream()), "gs_axpy");
    grid.newtonR1_ = false;
    grid.newtonVZero_ = false;
    return false;
}

// "[gs] mlups=... gbps=... pct_peak=... vcycle_ms=... cycles=... level_ms=a,b,..." over the V-cycles
// timed so far (GS_METRICS). mlups: level-0 smoother updates ((pre+post) x N0 per cycle) per second of
// V-cycle wall time; gbps: SURVEY.md §8(d)'s compulsory V-cycle traffic model, per level N_l points
// ((pre+post) x 24 B + 16 B residual/restriction + 16 B prolongation/correction + 2 B coarse, the
// coarsest level only its sweeps) + 16 B x N0 for the closing norm, per second; pct_peak against
// 8000 GB/s. level_ms: device time per level and cycle. Does not match runExperiments.py:46's regex.
std::string metricsLine(const HipGridData& grid)
{
    const LevelClock& c = grid.clock;
    if (c.cycles == 0) return "[gs] no V-cycle timed";
    const double ms = c.wallMs / c.cycles;
    const double sweeps = (double)(grid.preSmoothing + grid.postSmoothing);
    double bytes = 0.0;
    const std::size_t nl = grid.numLevels();
    for (std::size_t l = 0; l < nl; l++) {
        const auto& d = grid.getLevel(l).levelDim;
        const double n = (double)d[0] * (double)d[1] * (double)d[2];
        bytes += n * (sweeps * 24.0 + (l + 1 < nl ? 34.0 : 0.0));
    }
    const auto& d0 = grid.getLevel(0).levelDim;
    const double n0 = (double)d0[0] * (double)d0[1] * (double)d0[2];
    bytes += 16.0 * n0;
    const double gbps = bytes / (ms * 1e-3) / 1e9;
    char buf[256];
    std::snprintf(buf, sizeof buf, "[gs] mlups=%.1f gbps=%.1f pct_peak=%.1f vcycle_ms=%.3f cycles=%d level_ms=",
                  sweeps * n0 / (ms * 1e-3) / 1e6, gbps, 100.0 * gbps / 8000.0, ms, c.cycles);
    std::string out = buf;
    for (std::size_t l = 0; l < c.levelMs.size(); l++) {
        std::snprintf(buf, sizeof buf, "%s%.4f", l ? "," : "", c.levelMs[l] / c.cycles);
        out += buf;
    }
    return out;
}

void dumpField(HipGridData& grid, std::size_t level, const std::string& path)
{
    auto& L = grid.getLevel(level);
    HipSolver::materialize(grid, level);
    const gs_level& g = L.geom;
    const std::size_t px = (std::size_t)g.nx + 2, py = (std::size_t)g.ny + 2, pz = (std::size_t)g.nz + 2;
    std::vector<double> host(px * py * pz);
    check((int)hipStreamSynchronize(grid.stream()), "hipStreamSynchronize");
    check((int)hipMemcpy2D(host.data(), sizeof(double) * px, L.v.data(), sizeof(double) * (std::size_t)g.ldy,
                           sizeof(double) * px, py * pz, hipMemcpyDeviceToHost),
          "hipMemcpy2D");
    if (gs_dump_write(host.data(), (int64_t)px, (int64_t)py, (int64_t)pz, path.c_str()) != 0)
        throw Error(gs_last_error());
}

} // namespace gs
