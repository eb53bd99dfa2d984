// gs_grid.hpp — device-resident level hierarchy (HipGridData) and the V-cycle / Newton drivers.
//
// Mirrors the reference backend contract:
//   CpuGridData  (src/cpu/CpuGridData.{h,cpp})  -> gs::HipGridData
//   CpuSolver    (src/cpu/CpuSolver.{h,cpp})     -> gs::HipSolver   (solve, restrict public)
//   NewtonSolver (src/cpu/NewtonSolver.{h,cpp})  -> gs::NewtonSolver
// All fields live in HBM for the whole solve; the only device->host traffic per V-cycle is the
// 8-byte residual norm.
//
// Multi-GPU (new; the reference has none): with a Comm of size > 1 each level is either Z-slab
// partitioned (local planes + one ghost plane per side, kept current after every write of a field
// that is read with neighbours) or replicated below the agglomeration threshold.
#pragma once
#include <array>
#include <cstddef>
#include <cstdint>
#include <initializer_list>
#include <memory>
#include <string>
#include <functional>
#include <vector>

#include "gpusolve_hip.h"
#include "gs_comm.hpp"
#include "gs_params.hpp"

namespace gs {

void check(int code, const char* what); // throws gs::Error with gs_strerror(code)

// One padded fp64 field in the pitched x-fastest layout of include/gpusolve_hip.h.
class DeviceField {
public:
    DeviceField() = default;
    DeviceField(int64_t nx, int64_t ny, int64_t nz, hipStream_t s, bool dry = false); // zero-filled
    // dry: the layout without device memory (schedule tracing, HipGridData's trace mode)
    ~DeviceField();
    DeviceField(const DeviceField&) = delete;
    DeviceField& operator=(const DeviceField&) = delete;
    DeviceField(DeviceField&& o) noexcept { *this = std::move(o); }
    DeviceField& operator=(DeviceField&& o) noexcept;

    double* data() const { return origin_; }
    int64_t ldy() const { return ldy_; }
    int64_t ldz() const { return ldz_; }
    int64_t span() const { return span_; } // elements from origin covering every padded point
    explicit operator bool() const { return base_ != nullptr || dry_; }
    void zero(hipStream_t s);
    void swap(DeviceField& o) noexcept;

private:
    double* base_ = nullptr;
    double* origin_ = nullptr;
    int64_t ldy_ = 0, ldz_ = 0, span_ = 0, alloc_ = 0;
    bool dry_ = false;
};

// A plain device buffer of doubles (workspaces), grown on demand.
class DeviceBuf {
public:
    DeviceBuf() = default;
    ~DeviceBuf();
    DeviceBuf(const DeviceBuf&) = delete;
    DeviceBuf& operator=(const DeviceBuf&) = delete;
    double* get(int64_t elems); // at least elems doubles (reallocated when larger; contents not kept)
    int64_t size() const { return n_; }

private:
    double* p_ = nullptr;
    int64_t n_ = 0;
};

struct StreamGuard {
    hipStream_t s = nullptr;
    // high: the device's greatest stream priority (the exchange path: boundary planes, ghost copies)
    explicit StreamGuard(bool create = true, bool high = false);
    ~StreamGuard();
};

// Per-level device time of the V-cycles (GS_METRICS=1 when the grid is created): HIP events around every level's
// down-leg (smoothing, residual + restriction) and up-leg (prolongation + smoothing) work on the
// compute stream, read back after each cycle's norm sync. Off: no event is recorded.
struct LevelClock {
    bool on = false;
    int cycles = 0;
    double wallMs = 0.0;         // host wall time of the V-cycles (norm readbacks included)
    std::vector<double> levelMs; // device ms per level, summed over cycles
    std::vector<hipEvent_t> ev;  // ev[2k], ev[2k+1] bracket segment k of the current cycle
    std::vector<int> segLevel;   // level of segment k
    void mark(hipStream_t s, int level, bool begin);
    void collect();              // after a host sync: add this cycle's segments
    ~LevelClock();
};

class HipGridData final : public GridParams {
public:
    struct LevelData {
        DeviceField v;       // current iterate
        DeviceField vAlt;    // Jacobi ping-pong partner (the fused sweep reads v, writes vAlt)
        DeviceField restV;   // restricted v (FAS)
        DeviceField newtonV; // Newton linearisation point
        DeviceField newtonVNext; // (level 1, single GPU) R(level 0's newtonV) from the last compF update, swapped
                                 // in by the next findError — until then newtonV keeps the reference's value
        DeviceField f;       // right-hand side
        DeviceField r;       // residual (restriction source)
        DeviceField bfac;    // NEWTON (GS_NEWTON_B): B = gamma (1 + newtonV) exp(newtonV) of the inner solve's
                             // linearisation point, set by findError (gs_newton_bfac)
        std::array<std::size_t, 3> levelDim{}; // global interior extents
        double h = 0.0;
        gs_level geom{};     // kernel-side geometry of the stored array (slab or full level)
        bool distributed = false;
        bool fusedPairs = false; // smoothing runs as fused sweep pairs (gs_jacobi_sweep2)
        bool vZero = false;      // v is identically zero but not stored: the next sweep reads no v
        bool tiled = false;      // small LINEAR level: down- and up-leg steps as one tiled launch each
        int64_t lo = 1, hi = 0; // this rank's owned global planes (== 1..nz when not distributed)
        int64_t minPlanes = 0;  // fewest planes any rank owns on this level
        std::vector<int64_t> ranksLo, ranksHi; // every rank's owned planes (gather of replicated levels)
        // workspaces of the fused prolongation pair on column-block rows (gs_jacobi_sweep2_prolong_ws):
        // [0] for launches on the compute stream, [1] on the boundary stream (they run concurrently)
        std::unique_ptr<DeviceBuf[]> proWs = std::make_unique<DeviceBuf[]>(2);
    };

    // comm == nullptr or comm->size() == 1: the single-GPU path. The grid does not own comm.
    // trace != nullptr: schedule-trace mode — no device is touched; every kernel launch, ghost
    // exchange, gather, norm reduction, swap and zeroing the solvers would issue is appended to *trace
    // as one "op key=value ..." line instead (gs_zslab_schedule; replayed by tests/test_zslab_cpu.py
    // with the oracle's arithmetic on gloo ranks).
    explicit HipGridData(const GridParams& grid, Comm* comm = nullptr, int64_t agglomeratePoints = -1,
                         std::vector<std::string>* trace = nullptr);
    ~HipGridData();

    LevelData& getLevel(std::size_t l) { return levels_[l]; }
    const LevelData& getLevel(std::size_t l) const { return levels_[l]; }
    std::size_t numLevels() const { return levels_.size(); }

    DeviceField newtonF;  // Newton: the original right-hand side (src/cpu/CpuGridData.h:36)
    gs_stencil stencilAbi{};
    hipStream_t stream() const { return stream_.s; }
    hipStream_t commStream() const { return commStream_.s; }
    Comm* comm() const { return comm_; }
    int rank() const { return comm_ ? comm_->rank() : 0; }
    int nranks() const { return comm_ ? comm_->size() : 1; }
    bool overlapHalo = true; // boundary planes first, halo on the comm stream beside the interior
    // Alternative-path switches, read from the environment once, when the grid is created (never on a
    // launch path); the defaults are the measured choices. Tests pin every alternative bit-identical.
    struct Switches {
        bool fusedSweeps = true;   // GS_NO_FUSED_SWEEPS: one-sweep kernels only
        bool speculation = true;   // GS_NO_SPECULATION: the closing norm from a residual pass
        bool fusedProlong = true;  // GS_NO_FUSED_PROLONG: gs_prolong_add + the plain pair
        bool fusedRR = true;       // GS_NO_FUSED_RR: residual stored, then restricted
        bool zeroGuess = true;     // GS_NO_ZERO_GUESS: coarse v = 0 stored instead of flagged
        bool pipeline = true;      // GS_NO_PIPELINE: no overlap of the norm wait with the next cycle
        bool newtonFusedUpdate = true; // GS_NO_NEWTON_FUSED_UPDATE: newtonV += v, then compF (two passes)
        bool newtonB = true; // GS_NO_NEWTON_B: inner Newton solves read newtonV (GS_NEWTON) instead of the
                             // precomputed factor B (GS_NEWTON_B: exp(newtonV) once per point and Newton iteration)
        bool newtonBFused = true; // GS_NEWTON_B_FUSED=0: level 0's factor from its own gs_newton_bfac pass instead
                                  // of the compF update pass (bit-identical)
        bool newtonG = true; // GS_NO_NEWTON_G: the first Newton iteration's inner solve reads its factor fields (all
                             // gamma) instead of taking gamma in the pairs and k_rr2 (GS_NEWTON_G; bit-identical)
        int64_t tilePoints = (int64_t)1 << 18; // GS_TILE_POINTS: levels of at most this many points (replicated,
                                               // LINEAR) run the tiled one-launch down/up-leg steps; 0 = off
        int64_t newtonProPoints = (int64_t)1 << 21; // GS_NEWTON_PRO_POINTS: NEWTON levels take the fused
                                                     // prolongation pair from this many points per rank (r06: 2^21,
                                                     // 128^3 too, was 2^24)
        // GS_HALO_ORDER: in a pipelined Z-slab sweep sequence, interior k goes before boundary k when
        // exchange k-1 has not settled on the host yet (0, adaptive), always (1), or never (2: boundary first)
        int haloOrder = 0;
    } sw;
    // levels coarseFrom .. numLevels()-1 run as ONE gs_coarse_cycle launch in every V-cycle
    // (numLevels(): none); set from GS_COARSE_POINTS at construction
    std::size_t coarseFrom = 0;
    LevelClock clock; // per-level timing (GS_METRICS)
    std::vector<std::string>* trace = nullptr; // schedule-trace mode (see the constructor)
    void rec(const char* op, std::initializer_list<std::pair<const char*, long long>> kv, const char* field = nullptr);
    std::size_t levelIndex(const LevelData& L) const { return (std::size_t)(&L - levels_.data()); }
    static const char* fieldName(const LevelData& L, const DeviceField& f);

    // residual-norm plumbing: per-block partials, device scalars, pinned host scalar
    double* partials() const { return partials_; }
    double* dNorm() const { return dNorm_; }       // this rank's sum of squares (distributed norms)
    double* hNormDev() const { return hNormDev_; } // the pinned norm word, as the finishing kernel writes it
    double* dRankSums() const { return dRankSums_; }
    double readNorm(); // stream sync + the pinned norm word: the one host sync per V-cycle
    // the same in two halves: an event now, the (bounded) wait for the event later, so
    // that more work can be enqueued in between
    void readNormBegin();
    double readNormEnd();
    void sync();       // stream sync (bounded, error-polling when distributed over RCCL)

    // the mode and the w operand the V-cycle's kernels take: GS_NEWTON_B and B while findError's inner solve runs
    // with the factor fields current (newtonB_), else the grid's mode and newtonV (reference expressions)
    int kmode() const { return newtonB_ ? (bconst_ ? (int)GS_NEWTON_G : (int)GS_NEWTON_B) : (int)mode; }
    const double* wOf(const LevelData& L) const
    {
        return newtonB_ ? L.bfac.data() : (L.newtonV ? L.newtonV.data() : nullptr);
    }
    // newtonV may have been written from outside the solvers (the C ABI's writable field pointer or an upload):
    // nothing derived from it may be reused — not the zero-field shortcut (newtonVZero_), nor level 1's restriction
    // (newtonR1_) or level 0's factor (bfacFresh_) that the last update pass wrote
    void newtonVTouched()
    {
        newtonVZero_ = false;
        newtonR1_ = false;
        bfacFresh_ = 0;
    }
    // AND of `flag` over every rank of a distributed grid (an allgather of one word; the flag itself elsewhere), so
    // that a schedule decision taken from per-process state issues the same collectives on every rank
    bool allRanks(bool flag);
    // ghost planes of a distributed level's field (no-op otherwise); depth 2 where possible for
    // iterate fields (the fused pair reads two ghost planes of v)
    void halo(LevelData& L, DeviceField& fld, hipStream_t s, int depth = 1);
    // the same in halves (the pipelined sweep sequence, HipSolver::jacobi): haloIssue starts the exchange,
    // haloSettle() returns once its kernels are on s (only then may an event be recorded after it);
    // haloReady(): one poll of an issued exchange (trace mode: GS_HALO_ORDER decides, see Switches)
    void haloIssue(LevelData& L, DeviceField& fld, hipStream_t s, int depth);
    bool haloReady();
    void haloSettle();
    double haloHostMs = 0.0;    // host wall time spent issuing and settling ghost exchanges, summed
    double haloHostMaxMs = 0.0; // ... the largest for one exchange (issue + polls + settle)
    int64_t haloCalls = 0;
    int vDepth(const LevelData& L) const { return L.minPlanes >= 2 ? 2 : 1; }
    // replicated level fed from a distributed parent: assemble every rank's owned planes
    void gather(LevelData& L, DeviceField& fld);
    // geometry + pointer offset of the planes this rank computes on level L
    gs_level ownedGeom(const LevelData& L, int64_t* planeOffset) const;

private:
    std::vector<LevelData> levels_;
    Comm* comm_ = nullptr;
    StreamGuard stream_;
    StreamGuard commStream_;
    StreamGuard bndStream_; // boundary planes of an overlapped Z-slab sweep (distributed grids only)
    double* partials_ = nullptr;
    double* dNorm_ = nullptr;
    double* dRankSums_ = nullptr;
    double* hNorm_ = nullptr;
    double* hNormDev_ = nullptr;
    hipEvent_t evA_ = nullptr, evB_ = nullptr, evC_ = nullptr, evNorm_ = nullptr;
    hipEvent_t evBnd_[2] = {nullptr, nullptr}; // boundary planes of sweep k (k & 1) in a pipelined sequence
    std::vector<double> dryParts_;
    long traceNorms_ = 0;
    bool haloPending_ = false; // an exchange issued by haloIssue, not settled
    friend class NewtonSolver;
    bool newtonR1_ = false;    // level 1's newtonVNext holds R(level 0's newtonV) (gs_newton_F_update_restrict)
    bool newtonB_ = false;     // every level's bfac holds B of its current newtonV (set for the inner solve)
    bool bconst_ = false;      // ... and that B is gamma everywhere (newtonV = 0, the first iteration): GS_NEWTON_G
    unsigned bfacFresh_ = 0;   // bit l: level l's bfac already holds B of the newtonV the next findError uses
    bool newtonVZero_ = false; // every level's newtonV is still the zero of grid creation (the first findError)
    double haloCurMs_ = 0.0;   // host ms spent on that exchange so far
    double traceNorm();
    friend class HipSolver;
};

class HipSolver {
public:
    static void solve(HipGridData& grid);
    static void restrict(HipGridData& grid, const DeviceField& src, std::size_t srcLevel, DeviceField& dst);

    // exposed for benchmarks / the C ABI
    static double compResidual(HipGridData& grid, std::size_t level, bool storeR, bool norm);
    static double vcycle(HipGridData& grid);
    // The solve loop's V-cycle: with speculation on, a cycle's closing norm comes out of the first
    // pre-smoothing step of the next cycle (same residual, computed by that step anyway: one sweep
    // or a fused pair), run into vAlt without swapping; *pending = how many sweeps vAlt holds (0:
    // none), and the next cycle adopts them.
    static double vcycleSpeculative(HipGridData& grid, int* pending);
    // vcycleSpeculative in two halves: cycleDown enqueues everything that leaves level 0's iterate
    // untouched (adopting the pending speculative sweeps, every down-leg, the coarse end, the up-legs
    // of levels >= 1); cycleUp0 enqueues level 0's up-leg and the closing norm, and waits for the norm
    // only if `wait` (else the caller collects it with grid.readNormEnd()).
    static void cycleDown(HipGridData& grid, int* pending);
    static double cycleUp0(HipGridData& grid, int* pending, bool wait);
    // Up to maxCycles V-cycles with the host's wait for cycle i's norm overlapped with cycle i+1's
    // cycleDown (when pipelinable): onNorm(i, res) gets each closing norm in order and returns true
    // to stop — the early-enqueued work then only wrote coarse levels and scratch, and the adoption
    // of the speculative level-0 sweeps is undone, so level 0 holds cycle i's iterate exactly as
    // without the overlap. *pending: the speculative sweeps vAlt holds on entry and on return.
    // lastNormDead: the last cycle's closing norm is not computed (nobody reads it, see solve())
    static std::size_t runCycles(HipGridData& grid, int* pending, std::size_t maxCycles,
                                 const std::function<bool(std::size_t, double)>& onNorm, bool lastNormDead = false);
    static void cycleUpNoNorm(HipGridData& grid);
    static bool pipelinable(const HipGridData& grid, int pending);
    static void upLeg(HipGridData& grid, std::size_t level); // level-1 -> level-1 up-leg (from `level`)
    // level-0 sweep or pair v -> vAlt (no swap) + norm of f - A v; *sweeps = sweeps run; !wait: the
    // norm is left in flight (grid.readNormEnd())
    static double speculativeSweep(HipGridData& grid, int* sweeps, bool wait = true);
    static bool speculationEnabled(const HipGridData& grid);
    static void jacobi(HipGridData& grid, std::size_t level, std::size_t sweeps);
    static void materialize(HipGridData& grid, std::size_t level); // store a pending v = 0
    // the V-cycle below level `from` (its f set) in one gs_coarse_cycle launch
    static void coarseCycle(HipGridData& grid, std::size_t from);
    static double finishNorm(HipGridData& grid, int64_t nparts, bool wait = true);
    static hipStream_t forkBoundary(HipGridData& grid);
    static void forkComm(HipGridData& grid);
    static void joinComm(HipGridData& grid, bool wait);
    static void settleExchange(HipGridData& grid);

    // solve() records its residual history here when non-null (initial, then one per V-cycle)
    static thread_local std::vector<double>* history;
};

class NewtonSolver {
public:
    static void solve(HipGridData& grid);
    static double compF(HipGridData& grid);
    // findError's newtonV += v, left to compFUpdate when fusedUpdate() (returns whether it was deferred)
    static bool findError(HipGridData& grid);
    static double compFUpdate(HipGridData& grid);
    static bool fusedUpdate(const HipGridData& grid);
    static thread_local std::vector<double>* history;
};

// The optional machine-readable metrics line of GpuSolve-hip (GS_METRICS=1), see gs_grid.cpp.
std::string metricsLine(const HipGridData& grid);

// Vector3::dump (src/cpu/Vector3.cpp:56-78) of level `level`'s iterate v (this rank's slab).
void dumpField(HipGridData& grid, std::size_t level, const std::string& path);

} // namespace gs
