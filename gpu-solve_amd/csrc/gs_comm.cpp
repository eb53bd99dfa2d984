// gs_comm.cpp — Z-slab plan, RCCL communicator, single-device loopback communicator.
#include "gs_comm.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include <unistd.h>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "gs_params.hpp"

namespace gs {

namespace {
// RCCL's workgroups per exchange group (ncclConfig_t::minCTAs = maxCTAs; GS_RCCL_CTAS overrides): the
// stand-in exchange at RCCL's kernel footprint (34 MB per step) finishes the overlapped config #5 slab step
// sooner with more workgroups — 0.958 / 0.838 / 0.826 / 0.771-0.789 / 0.752-0.754 ms at 8 / 16 / 32 / 64 / 128
// against 0.722 ms without an exchange (profiles/r04/r04b_exchange_wgs.json); 64 is NCCL's channel limit
constexpr int kRcclCtasDefault = 64;

void hipOk(hipError_t e, const char* what)
{
    if (e != hipSuccess) throw Error(std::string(what) + ": " + hipGetErrorString(e));
}
void ncclOk(ncclResult_t e, const char* what)
{
    if (e != ncclSuccess) throw Error(std::string(what) + ": " + ncclGetErrorString(e));
}
} // namespace

// ---------------------------------------------------------------------------------------------
void Comm::sync(hipStream_t s) { hipOk(hipStreamSynchronize(s), "hipStreamSynchronize"); }
void Comm::syncEvent(hipEvent_t e) { hipOk(hipEventSynchronize(e), "hipEventSynchronize"); }

// RCCL over xGMI: halo planes are point-to-point send/recv with the two z-neighbours, grouped so
// each rank's four operations progress together; the norm is an all-gather of one double. The
// communicator is non-blocking so that no call can hang the host past its deadline: each call (or
// group) is settled by polling ncclCommGetAsyncError, and sync() polls it beside hipStreamQuery.
class RcclComm final : public Comm {
public:
    RcclComm(int rank, int nranks, const void* uid, int ctas) : r_(rank), n_(nranks), ctas_(ctas)
    {
        const char* inj = std::getenv("GS_COMM_INJECT_ERROR");
        injectAt_ = inj ? std::atol(inj) : 0;
        timeout_ = commTimeoutS("GS_COMM_TIMEOUT_S", 120.0);
        ncclUniqueId id;
        std::memcpy(&id, uid, sizeof(id));
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        if (ctas_ > 0) {
            // the CTA budget caps RCCL's send/recv grid; the p2p channels per peer fill it (a rank's grouped
            // exchange is four send/recv operations, so NCCL_NCHANNELS_PER_PEER = ctas / 4 gives it the whole
            // budget: profiles/r04/r04i_rccl_grid_cpp16.txt). RCCL reads that variable once per process, so
            // the LAUNCHER sets it before any communicator exists (GpuSolve-hip's main, bench.py;
            // rcclChannelsPerPeerHint); the library never writes the process environment
            cfg.minCTAs = ctas_;
            cfg.maxCTAs = ctas_;
        }
        const ncclResult_t e = ncclCommInitRankConfig(&c_, nranks, id, rank, &cfg);
        if (e != ncclSuccess && e != ncclInProgress) {
            if (c_) (void)ncclCommAbort(c_);
            c_ = nullptr;
            fail("ncclCommInitRankConfig", ncclGetErrorString(e));
        }
        settle("ncclCommInitRankConfig", commTimeoutS("GS_COMM_INIT_TIMEOUT_S", 300.0));
    }
    ~RcclComm() override
    {
        if (c_) (void)ncclCommDestroy(c_);
    }
    int rank() const override { return r_; }
    int size() const override { return n_; }

    void halo(double* field, int64_t ldz, int64_t nzl, int depth, hipStream_t s) override
    {
        haloIssue(field, ldz, nzl, depth, s);
        haloSettle();
    }

    void haloIssue(double* field, int64_t ldz, int64_t nzl, int depth, hipStream_t s) override
    {
        haloSettle(); // (one exchange in flight at a time)
        if (n_ == 1) return;
        const size_t cnt = (size_t)(depth * ldz);
        call(ncclGroupStart(), "ncclGroupStart");
        if (r_ > 0) {
            call(ncclSend(field + ldz, cnt, ncclDouble, r_ - 1, c_, s), "ncclSend");
            call(ncclRecv(field + (1 - depth) * ldz, cnt, ncclDouble, r_ - 1, c_, s), "ncclRecv");
        }
        if (r_ + 1 < n_) {
            call(ncclSend(field + (nzl - depth + 1) * ldz, cnt, ncclDouble, r_ + 1, c_, s), "ncclSend");
            call(ncclRecv(field + (nzl + 1) * ldz, cnt, ncclDouble, r_ + 1, c_, s), "ncclRecv");
        }
        call(ncclGroupEnd(), "ncclGroupEnd");
        pending_ = true;
        // counted here, once per exchange, whichever of haloReady / haloSettle completes it
        pendingInject_ = injectNow();
    }

    bool haloReady() override
    {
        if (!pending_) return true;
        const int a = asyncState(pendingInject_);
        if (a > 1) abortAndThrow(std::string("halo exchange: ") + ncclGetErrorString((ncclResult_t)(a - 2)));
        if (a == 0) pending_ = false;
        return !pending_;
    }

    void haloSettle() override
    {
        if (!pending_) return;
        pending_ = false;
        settleAs("halo exchange", timeout_, pendingInject_);
    }
    int ctas() const override { return ctas_; }

    void allgather1(const double* in, double* out, hipStream_t s) override
    {
        haloSettle();
        call(ncclAllGather(in, out, 1, ncclDouble, c_, s), "ncclAllGather");
        settle("ncclAllGather", timeout_);
    }

    void gatherPlanes(double* field, int64_t ldz, const std::vector<int64_t>& lo, const std::vector<int64_t>& hi,
                      hipStream_t s) override
    {
        haloSettle();
        call(ncclGroupStart(), "ncclGroupStart");
        for (int q = 0; q < n_; q++) {
            if (hi[q] < lo[q]) continue;
            double* p = field + lo[q] * ldz;
            call(ncclBroadcast(p, p, (size_t)((hi[q] - lo[q] + 1) * ldz), ncclDouble, q, c_, s), "ncclBroadcast");
        }
        call(ncclGroupEnd(), "ncclGroupEnd");
        settle("plane gather", timeout_);
    }

    void sync(hipStream_t s) override
    {
        haloSettle();
        wait([&] { return hipStreamQuery(s); }, "stream sync");
    }
    void syncEvent(hipEvent_t e) override
    {
        haloSettle();
        wait([&] { return hipEventQuery(e); }, "event sync");
    }

private:
    // a bounded wait for `query` (hipStreamQuery / hipEventQuery) that polls the async error state
    void wait(const std::function<hipError_t()>& query, const char* what)
    {
        const bool inject = injectNow();
        const std::string err = boundedWait(
            [&]() -> int {
                const hipError_t q = query();
                const int a = asyncState(inject);
                if (a > 1) return a;
                if (q == hipSuccess) return 0;
                if (q != hipErrorNotReady) return -(int)q;
                return 1;
            },
            [](int st) {
                return st < 0 ? std::string(hipGetErrorString((hipError_t)-st))
                              : std::string(ncclGetErrorString((ncclResult_t)(st - 2)));
            },
            timeout_, what);
        if (!err.empty()) abortAndThrow(err);
    }

    // 1 in progress, 0 settled, 2 + ncclResult_t for an error
    int asyncState(bool inject)
    {
        ncclResult_t a = ncclSuccess;
        const ncclResult_t e = ncclCommGetAsyncError(c_, &a);
        if (e != ncclSuccess) a = e;
        if (inject) a = ncclInternalError;
        if (a == ncclSuccess) return 0;
        if (a == ncclInProgress) return 1;
        return 2 + (int)a;
    }
    void call(ncclResult_t e, const char* what)
    {
        if (e != ncclSuccess && e != ncclInProgress) abortAndThrow(std::string(what) + ": " + ncclGetErrorString(e));
    }
    // GS_COMM_INJECT_ERROR=k: the k-th settle / sync of this communicator sees ncclInternalError (an
    // exchange counts once, when it is issued: haloIssue)
    bool injectNow() { return injectAt_ > 0 && ++calls_ == injectAt_; }
    void settle(const char* what, double timeoutS) { settleAs(what, timeoutS, injectNow()); }
    void settleAs(const char* what, double timeoutS, bool inject)
    {
        const std::string err = boundedWait(
            [&] { return asyncState(inject); },
            [](int st) { return std::string(ncclGetErrorString((ncclResult_t)(st - 2))); }, timeoutS, what);
        if (!err.empty()) abortAndThrow(err);
    }
    [[noreturn]] void abortAndThrow(const std::string& msg)
    {
        if (c_) (void)ncclCommAbort(c_);
        c_ = nullptr;
        fail("RCCL", msg.c_str());
    }
    [[noreturn]] void fail(const char* what, const char* msg) const
    {
        throw Error(std::string(what) + " " + msg + " (rank " + std::to_string(r_) + " of " + std::to_string(n_) +
                    "); communicator aborted");
    }
    int r_, n_, ctas_;
    ncclComm_t c_ = nullptr;
    long injectAt_ = 0, calls_ = 0;
    double timeout_ = 120.0;
    bool pending_ = false;       // an issued halo exchange not yet settled
    bool pendingInject_ = false; // GS_COMM_INJECT_ERROR picked that exchange
};

int rcclCtas()
{
    static const int n = [] {
        const char* e = std::getenv("GS_RCCL_CTAS");
        return e && *e ? std::max(0, std::atoi(e)) : kRcclCtasDefault;
    }();
    return n;
}

std::unique_ptr<Comm> makeRcclComm(int rank, int nranks, const void* uid, int ctas)
{
    return std::make_unique<RcclComm>(rank, nranks, uid, ctas < 0 ? rcclCtas() : ctas);
}

int rcclChannelsPerPeerHint(int ctas)
{
    if (ctas < 0) ctas = rcclCtas();
    return ctas > 0 ? std::max(1, ctas / 4) : 0;
}

void rcclUniqueId(void* uid)
{
    ncclUniqueId id;
    ncclOk(ncclGetUniqueId(&id), "ncclGetUniqueId");
    std::memcpy(uid, &id, sizeof(id));
}

// ---------------------------------------------------------------------------------------------
// Loopback: N ranks = N host threads on one device. A rank publishes its buffer and an event
// recorded after the producing work; after a host barrier every rank makes its stream wait on
// the producers' events and copies device-to-device, then records a "consumed" event that the
// producers' streams wait on before they may overwrite the planes. Same ordering contract as RCCL
// send/recv, so the Z-slab solver is exercised unchanged on one GPU.
void abortLoopbackHub(LoopbackHub& hub, const std::string& why) { hub.abort(why); }
std::string loopbackHubError(LoopbackHub& hub) { return hub.error(); }
void loopbackHubBarrier(LoopbackHub& hub) { hub.barrier(); }

std::shared_ptr<LoopbackHub> makeLoopbackHub(int nranks) { return std::make_shared<LoopbackHub>(nranks); }

class LoopbackComm final : public Comm {
public:
    LoopbackComm(std::shared_ptr<LoopbackHub> hub, int rank) : h_(std::move(hub)), r_(rank)
    {
        auto& me = h_->slots_[r_];
        hipEvent_t a = nullptr, b = nullptr;
        hipOk(hipEventCreateWithFlags(&a, hipEventDisableTiming), "hipEventCreate");
        hipOk(hipEventCreateWithFlags(&b, hipEventDisableTiming), "hipEventCreate");
        me.produced = a;
        me.consumed = b;
    }
    ~LoopbackComm() override
    {
        auto& me = h_->slots_[r_];
        if (me.produced) (void)hipEventDestroy((hipEvent_t)me.produced);
        if (me.consumed) (void)hipEventDestroy((hipEvent_t)me.consumed);
    }
    int rank() const override { return r_; }
    int size() const override { return h_->n_; }

    void halo(double* field, int64_t ldz, int64_t nzl, int depth, hipStream_t s) override
    {
        publish(field, ldz, nzl, s);
        const size_t bytes = sizeof(double) * (size_t)(depth * ldz);
        if (r_ > 0) { // rank-1's planes nzl'-depth+1 .. nzl' -> my planes 1-depth .. 0
            auto& nb = h_->slots_[r_ - 1];
            hipOk(hipStreamWaitEvent(s, (hipEvent_t)nb.produced, 0), "hipStreamWaitEvent");
            hipOk(hipMemcpyAsync(field + (1 - depth) * ldz, nb.p + (nb.b - depth + 1) * ldz, bytes,
                                 hipMemcpyDeviceToDevice, s),
                  "hipMemcpyAsync");
        }
        if (r_ + 1 < size()) { // rank+1's planes 1 .. depth -> my planes nzl+1 .. nzl+depth
            auto& nb = h_->slots_[r_ + 1];
            hipOk(hipStreamWaitEvent(s, (hipEvent_t)nb.produced, 0), "hipStreamWaitEvent");
            hipOk(hipMemcpyAsync(field + (nzl + 1) * ldz, nb.p + ldz, bytes, hipMemcpyDeviceToDevice, s),
                  "hipMemcpyAsync");
        }
        release(s, r_ > 0 ? r_ - 1 : -1, r_ + 1 < size() ? r_ + 1 : -1);
    }

    void allgather1(const double* in, double* out, hipStream_t s) override
    {
        publish(in, 0, 0, s);
        for (int q = 0; q < size(); q++) {
            auto& nb = h_->slots_[q];
            hipOk(hipStreamWaitEvent(s, (hipEvent_t)nb.produced, 0), "hipStreamWaitEvent");
            hipOk(hipMemcpyAsync(out + q, nb.p, sizeof(double), hipMemcpyDeviceToDevice, s), "hipMemcpyAsync");
        }
        release(s, -2, -2);
    }

    void gatherPlanes(double* field, int64_t ldz, const std::vector<int64_t>& lo, const std::vector<int64_t>& hi,
                      hipStream_t s) override
    {
        publish(field, ldz, 0, s);
        for (int q = 0; q < size(); q++) {
            if (q == r_ || hi[q] < lo[q]) continue;
            auto& nb = h_->slots_[q];
            hipOk(hipStreamWaitEvent(s, (hipEvent_t)nb.produced, 0), "hipStreamWaitEvent");
            hipOk(hipMemcpyAsync(field + lo[q] * ldz, nb.p + lo[q] * ldz,
                                 sizeof(double) * (size_t)((hi[q] - lo[q] + 1) * ldz), hipMemcpyDeviceToDevice, s),
                  "hipMemcpyAsync");
        }
        release(s, -2, -2);
    }

private:
    void publish(const double* p, int64_t a, int64_t b, hipStream_t s)
    {
        auto& me = h_->slots_[r_];
        me.p = p;
        me.a = a;
        me.b = b;
        hipOk(hipEventRecord((hipEvent_t)me.produced, s), "hipEventRecord");
        h_->barrier();
    }
    // q1/q2: the ranks that read our buffer (-2: everyone)
    void release(hipStream_t s, int q1, int q2)
    {
        auto& me = h_->slots_[r_];
        hipOk(hipEventRecord((hipEvent_t)me.consumed, s), "hipEventRecord");
        h_->barrier();
        for (int q = 0; q < size(); q++) {
            if (q == r_) continue;
            if (q1 != -2 && q != q1 && q != q2) continue;
            hipOk(hipStreamWaitEvent(s, (hipEvent_t)h_->slots_[q].consumed, 0), "hipStreamWaitEvent");
        }
        h_->barrier();
    }
    std::shared_ptr<LoopbackHub> h_;
    int r_;
};

class TraceComm final : public Comm {
public:
    TraceComm(int rank, int n) : r_(rank), n_(n) {}
    int rank() const override { return r_; }
    int size() const override { return n_; }
    void halo(double*, int64_t, int64_t, int, hipStream_t) override { throw Error("trace communicator: no transport"); }
    void allgather1(const double*, double*, hipStream_t) override { throw Error("trace communicator: no transport"); }
    void gatherPlanes(double*, int64_t, const std::vector<int64_t>&, const std::vector<int64_t>&, hipStream_t) override
    {
        throw Error("trace communicator: no transport");
    }
    void sync(hipStream_t) override {}
    void syncEvent(hipEvent_t) override {}

private:
    int r_, n_;
};

std::unique_ptr<Comm> makeTraceComm(int rank, int nranks) { return std::make_unique<TraceComm>(rank, nranks); }

std::unique_ptr<Comm> makeLoopbackComm(const std::shared_ptr<LoopbackHub>& hub, int rank)
{
    return std::make_unique<LoopbackComm>(hub, rank);
}

} // namespace gs
