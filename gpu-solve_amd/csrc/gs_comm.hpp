// gs_comm.hpp — the exchange layer of the Z-slab decomposition.
//
// The reference has no distributed path; this is new. A level of the hierarchy is either
// Z-slab-partitioned (rank r owns the contiguous global interior planes [lo[r], hi[r]] plus one
// ghost plane on each side) or replicated (every rank holds the full level and computes it
// redundantly; used below the agglomeration threshold). Everything a rank needs from another one is:
//   halo()          its z-neighbours' boundary planes (send/recv of one padded plane each way),
//   allgather1()    one double per rank (the l2-norm partial sums; summed in rank order after),
//   gatherPlanes()  the owned planes of a replicated level, assembled on every rank.
// Implementations: RCCL over xGMI (one process per GPU, or one thread per GPU), and a loopback that
// runs N ranks as N threads on one device with device-to-device copies (tests on a single GPU).
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "gs_hostsync.hpp"

namespace gs {

class Comm {
public:
    virtual ~Comm() = default;
    virtual int rank() const = 0;
    virtual int size() const = 0;
    // field: padded plane p of this rank's slab at field + p*ldz, local interior planes 1..nzl.
    // depth 1: sends plane 1 to rank-1 and plane nzl to rank+1; receives rank-1's top plane into
    // plane 0 and rank+1's bottom plane into plane nzl+1. depth 2 (nzl >= 2): the two outermost
    // planes each way, into planes -1..0 and nzl+1..nzl+2. Asynchronous on s.
    virtual void halo(double* field, int64_t ldz, int64_t nzl, int depth, hipStream_t s) = 0;
    // halo() in two halves, for RCCL's non-blocking group: haloIssue() starts the exchange and returns;
    // its kernels are on s once haloSettle() has returned (the communicator settles a pending exchange
    // itself before any other call). haloReady(): one poll, true once it has settled. Work that must
    // follow the exchange on s (an event record) is enqueued only after haloSettle(). The default
    // (loopback, trace) settles inside haloIssue().
    virtual void haloIssue(double* field, int64_t ldz, int64_t nzl, int depth, hipStream_t s)
    {
        halo(field, ldz, nzl, depth, s);
    }
    virtual bool haloReady() { return true; }
    virtual void haloSettle() {}
    // out[r] <- rank r's *in, on every rank (out holds size() doubles). Asynchronous on s.
    virtual void allgather1(const double* in, double* out, hipStream_t s) = 0;
    // field: a full-size level on every rank; rank r has computed planes [lo[r], hi[r]]; afterwards
    // every rank holds every rank's planes. Asynchronous on s.
    virtual void gatherPlanes(double* field, int64_t ldz, const std::vector<int64_t>& lo, const std::vector<int64_t>& hi,
                              hipStream_t s) = 0;
    // Waits until everything enqueued on s has completed. The RCCL communicator bounds the wait and
    // polls the communicator's asynchronous error state while it waits: a dead or deadlocked peer
    // becomes a gs::Error (communicator aborted) instead of a hang. The solver's one host sync per
    // V-cycle (the norm readback) goes through here.
    virtual void sync(hipStream_t s);
    // The same wait for one event (work enqueued on the stream after it is not waited for).
    virtual void syncEvent(hipEvent_t e);
    // RCCL: the communicator's CTA budget (ncclConfig_t::minCTAs = maxCTAs; 0: RCCL's own); -1 otherwise
    virtual int ctas() const { return -1; }
};

// RCCL (NCCL API); uid is the 128-byte ncclUniqueId created by rank 0 (rcclUniqueId) and shared.
// The communicator is non-blocking (ncclConfig_t::blocking = 0): initialisation and every grouped
// call are settled by polling ncclCommGetAsyncError under a deadline (GS_COMM_INIT_TIMEOUT_S, default
// 300 s; GS_COMM_TIMEOUT_S, default 120 s, also for sync()). On an error or a timeout the communicator
// is aborted (ncclCommAbort) and gs::Error("RCCL ... (rank r of n)") is thrown. GS_COMM_INJECT_ERROR=k
// (tests) makes the k-th settle or sync of the communicator see ncclInternalError (a halo exchange counts
// once, at its issue). ctas sets ncclConfig_t::minCTAs = maxCTAs: the workgroups RCCL's kernels take for a
// send/recv group, which share the CUs with the interior sweep they overlap (0: RCCL's own choice; -1: the
// process default rcclCtas()).
std::unique_ptr<Comm> makeRcclComm(int rank, int nranks, const void* uid, int ctas = -1);
// the process default CTA budget (GS_RCCL_CTAS, read once, else 64; 0: RCCL's)
int rcclCtas();
// NCCL_NCHANNELS_PER_PEER that gives a grouped exchange (four send/recv per rank) the whole budget `ctas`
// (-1: rcclCtas()): ctas / 4, 0 for RCCL's default. RCCL reads the variable once per process, so a LAUNCHER
// (GpuSolve-hip's main, bench.py) sets it, unless already set, before its first communicator; the library
// itself never writes the environment.
int rcclChannelsPerPeerHint(int ctas = -1);
void rcclUniqueId(void* uid);

// The rank-0 id file hand-off (publishUid / awaitUid / uidPath), the bounded wait and the loopback
// hub live in the HIP-free gs_hostsync.hpp.

// Rank `rank` of `nranks` without any transport: the communicator of HipGridData's schedule-trace
// mode, which records exchanges instead of running them.
std::unique_ptr<Comm> makeTraceComm(int rank, int nranks);

// Loopback: nranks threads of one process on one device share a hub (gs_hostsync.hpp).
std::shared_ptr<LoopbackHub> makeLoopbackHub(int nranks);
std::unique_ptr<Comm> makeLoopbackComm(const std::shared_ptr<LoopbackHub>& hub, int rank);
// A rank that fails calls this: every thread parked in (or later reaching) a hub barrier throws, so
// all rank threads unwind instead of waiting forever. loopbackHubError: the first message ("" = none).
void abortLoopbackHub(LoopbackHub& hub, const std::string& why);
std::string loopbackHubError(LoopbackHub& hub);
void loopbackHubBarrier(LoopbackHub& hub); // throws once the hub is aborted

// Plane ownership of every level (pure host logic).
struct SlabPlan {
    std::vector<char> distributed;            // per level
    std::vector<std::vector<int64_t>> lo, hi; // [level][rank], 1-based global interior planes
};
// levelNz: global interior planes per level; a level stays partitioned while its parent is,
// it is not the coarsest, every rank keeps >= 1 plane and its global point count is >= minPoints.
SlabPlan planZSlabs(const std::vector<int64_t>& levelNz, const std::vector<int64_t>& levelPoints, int nranks,
                    int64_t minPoints);

} // namespace gs
