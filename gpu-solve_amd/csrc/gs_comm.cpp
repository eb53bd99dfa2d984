// gs_comm.cpp — Z-slab plan, RCCL communicator, single-device loopback communicator.
#include "gs_comm.hpp"

#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "gs_params.hpp"

namespace gs {

namespace {
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
SlabPlan planZSlabs(const std::vector<int64_t>& levelNz, const std::vector<int64_t>& levelPoints, int nranks,
                    int64_t minPoints)
{
    const size_t L = levelNz.size();
    SlabPlan p;
    p.distributed.assign(L, 0);
    p.lo.assign(L, std::vector<int64_t>(nranks, 1));
    p.hi.assign(L, std::vector<int64_t>(nranks, 0));
    bool parent = nranks > 1;
    for (size_t l = 0; l < L; l++) {
        bool nonEmpty = true;
        for (int r = 0; r < nranks; r++) {
            if (l == 0) {
                p.lo[0][r] = 1 + (int64_t)r * levelNz[0] / nranks;
                p.hi[0][r] = (int64_t)(r + 1) * levelNz[0] / nranks;
            } else {
                p.lo[l][r] = (p.lo[l - 1][r] + 1) / 2; // coarse plane zc owned iff 2 zc is owned
                p.hi[l][r] = p.hi[l - 1][r] / 2;
            }
            nonEmpty = nonEmpty && p.hi[l][r] >= p.lo[l][r];
        }
        const bool dist = parent && nonEmpty && l + 1 < L && (l == 0 || levelPoints[l] >= minPoints);
        p.distributed[l] = dist;
        parent = dist;
    }
    return p;
}

// ---------------------------------------------------------------------------------------------
// RCCL over xGMI: halo planes are point-to-point send/recv with the two z-neighbours, grouped so
// each rank's four operations progress together; the norm is an all-gather of one double.
class RcclComm final : public Comm {
public:
    RcclComm(int rank, int nranks, const void* uid) : r_(rank), n_(nranks)
    {
        ncclUniqueId id;
        std::memcpy(&id, uid, sizeof(id));
        ncclOk(ncclCommInitRank(&c_, nranks, id, rank), "ncclCommInitRank");
    }
    ~RcclComm() override
    {
        if (c_) (void)ncclCommDestroy(c_);
    }
    int rank() const override { return r_; }
    int size() const override { return n_; }

    void halo(double* field, int64_t ldz, int64_t nzl, int depth, hipStream_t s) override
    {
        if (n_ == 1) return;
        const size_t cnt = (size_t)(depth * ldz);
        ncclOk(ncclGroupStart(), "ncclGroupStart");
        if (r_ > 0) {
            ncclOk(ncclSend(field + ldz, cnt, ncclDouble, r_ - 1, c_, s), "ncclSend");
            ncclOk(ncclRecv(field + (1 - depth) * ldz, cnt, ncclDouble, r_ - 1, c_, s), "ncclRecv");
        }
        if (r_ + 1 < n_) {
            ncclOk(ncclSend(field + (nzl - depth + 1) * ldz, cnt, ncclDouble, r_ + 1, c_, s), "ncclSend");
            ncclOk(ncclRecv(field + (nzl + 1) * ldz, cnt, ncclDouble, r_ + 1, c_, s), "ncclRecv");
        }
        ncclOk(ncclGroupEnd(), "ncclGroupEnd");
    }

    void allgather1(const double* in, double* out, hipStream_t s) override
    {
        ncclOk(ncclAllGather(in, out, 1, ncclDouble, c_, s), "ncclAllGather");
    }

    void gatherPlanes(double* field, int64_t ldz, const std::vector<int64_t>& lo, const std::vector<int64_t>& hi,
                      hipStream_t s) override
    {
        ncclOk(ncclGroupStart(), "ncclGroupStart");
        for (int q = 0; q < n_; q++) {
            if (hi[q] < lo[q]) continue;
            double* p = field + lo[q] * ldz;
            ncclOk(ncclBroadcast(p, p, (size_t)((hi[q] - lo[q] + 1) * ldz), ncclDouble, q, c_, s), "ncclBroadcast");
        }
        ncclOk(ncclGroupEnd(), "ncclGroupEnd");
    }

private:
    int r_, n_;
    ncclComm_t c_ = nullptr;
};

std::unique_ptr<Comm> makeRcclComm(int rank, int nranks, const void* uid)
{
    return std::make_unique<RcclComm>(rank, nranks, uid);
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
class LoopbackHub {
public:
    explicit LoopbackHub(int n) : n_(n), slots_(n) {}
    struct Slot {
        const double* p = nullptr;
        int64_t a = 0, b = 0;
        hipEvent_t produced = nullptr, consumed = nullptr;
    };
    void barrier()
    {
        std::unique_lock<std::mutex> lk(m_);
        const int gen = gen_;
        if (++count_ == n_) {
            count_ = 0;
            gen_++;
            cv_.notify_all();
        } else {
            cv_.wait(lk, [&] { return gen != gen_; });
        }
    }
    int n_;
    std::vector<Slot> slots_;

private:
    std::mutex m_;
    std::condition_variable cv_;
    int count_ = 0, gen_ = 0;
};

std::shared_ptr<LoopbackHub> makeLoopbackHub(int nranks) { return std::make_shared<LoopbackHub>(nranks); }

class LoopbackComm final : public Comm {
public:
    LoopbackComm(std::shared_ptr<LoopbackHub> hub, int rank) : h_(std::move(hub)), r_(rank)
    {
        auto& me = h_->slots_[r_];
        hipOk(hipEventCreateWithFlags(&me.produced, hipEventDisableTiming), "hipEventCreate");
        hipOk(hipEventCreateWithFlags(&me.consumed, hipEventDisableTiming), "hipEventCreate");
    }
    ~LoopbackComm() override
    {
        auto& me = h_->slots_[r_];
        if (me.produced) (void)hipEventDestroy(me.produced);
        if (me.consumed) (void)hipEventDestroy(me.consumed);
    }
    int rank() const override { return r_; }
    int size() const override { return h_->n_; }

    void halo(double* field, int64_t ldz, int64_t nzl, int depth, hipStream_t s) override
    {
        publish(field, ldz, nzl, s);
        const size_t bytes = sizeof(double) * (size_t)(depth * ldz);
        if (r_ > 0) { // rank-1's planes nzl'-depth+1 .. nzl' -> my planes 1-depth .. 0
            auto& nb = h_->slots_[r_ - 1];
            hipOk(hipStreamWaitEvent(s, nb.produced, 0), "hipStreamWaitEvent");
            hipOk(hipMemcpyAsync(field + (1 - depth) * ldz, nb.p + (nb.b - depth + 1) * ldz, bytes,
                                 hipMemcpyDeviceToDevice, s),
                  "hipMemcpyAsync");
        }
        if (r_ + 1 < size()) { // rank+1's planes 1 .. depth -> my planes nzl+1 .. nzl+depth
            auto& nb = h_->slots_[r_ + 1];
            hipOk(hipStreamWaitEvent(s, nb.produced, 0), "hipStreamWaitEvent");
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
            hipOk(hipStreamWaitEvent(s, nb.produced, 0), "hipStreamWaitEvent");
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
            hipOk(hipStreamWaitEvent(s, nb.produced, 0), "hipStreamWaitEvent");
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
        hipOk(hipEventRecord(me.produced, s), "hipEventRecord");
        h_->barrier();
    }
    // q1/q2: the ranks that read our buffer (-2: everyone)
    void release(hipStream_t s, int q1, int q2)
    {
        auto& me = h_->slots_[r_];
        hipOk(hipEventRecord(me.consumed, s), "hipEventRecord");
        h_->barrier();
        for (int q = 0; q < size(); q++) {
            if (q == r_) continue;
            if (q1 != -2 && q != q1 && q != q2) continue;
            hipOk(hipStreamWaitEvent(s, h_->slots_[q].consumed, 0), "hipStreamWaitEvent");
        }
        h_->barrier();
    }
    std::shared_ptr<LoopbackHub> h_;
    int r_;
};

std::unique_ptr<Comm> makeLoopbackComm(const std::shared_ptr<LoopbackHub>& hub, int rank)
{
    return std::make_unique<LoopbackComm>(hub, rank);
}

} // namespace gs
