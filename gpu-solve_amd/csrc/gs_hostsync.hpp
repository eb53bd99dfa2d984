// gs_hostsync.hpp — the HIP-free host logic of the exchange layer (gs_comm.hpp): the bounded wait that
// settles every RCCL call, the rank-0 id file hand-off, and the loopback hub's barrier/abort. Kept in
// its own translation unit (gs_hostsync.cpp) so the host sanitizer harnesses (oracle/Makefile: asan,
// tsan) build it without the HIP runtime.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

namespace gs {

// poll() returns 0 done, 1 still pending, or any other value = an error whose text errText(value)
// gives. Returns "" on completion, else the error / timeout message.
std::string boundedWait(const std::function<int()>& poll, const std::function<std::string(int)>& errText,
                        double timeoutS, const char* what);
double commTimeoutS(const char* env, double dflt);

// Sharing rank 0's 128-byte id between the processes of one node without another library (GpuSolve-hip
// under torchrun): rank 0 writes it to `path` (a temporary file renamed into place, so a reader sees
// all 128 bytes or nothing), the other ranks poll for it up to timeoutS (gs::Error on timeout).
void publishUid(const std::string& path, const unsigned char* uid);
void awaitUid(const std::string& path, double timeoutS, unsigned char* uid);
// $GS_UID_FILE, else /tmp/gpusolve-uid-<parent pid>-<$MASTER_PORT>[-<$TORCHELASTIC_RUN_ID>-
// <$TORCHELASTIC_RESTART_COUNT>]: the local ranks of one launcher share its pid, and each restart
// attempt of a torchrun agent (same pid, same port) gets its own file, so a file left behind by an
// attempt whose rank 0 was killed is never read by the next one.
std::string uidPath();

// Loopback: N ranks = N host threads on one device. The hub holds each rank's published buffer and
// events (opaque here) and the host barrier the ranks meet at; abort() wakes every waiting thread.
class LoopbackHub {
public:
    explicit LoopbackHub(int n) : n_(n), slots_(n) {}
    struct Slot {
        const double* p = nullptr;
        int64_t a = 0, b = 0;
        void* produced = nullptr; // hipEvent_t (gs_comm.cpp)
        void* consumed = nullptr;
    };
    void barrier(); // throws gs::Error once the hub is aborted
    void abort(const std::string& why);
    std::string error();
    int n_;
    std::vector<Slot> slots_;

private:
    std::mutex m_;
    std::condition_variable cv_;
    int count_ = 0, gen_ = 0;
    bool aborted_ = false;
    std::string why_;
};

// Self-tests of the above (gs_debug_* in the C ABI, and the sanitizer harnesses):
// scenario 0 completes at poll k, 1 reports an error at poll k, 2 never completes.
int debugBoundedWait(int scenario, int k, double timeoutS, std::string* msg);
// nranks threads meet at hub barriers and failing_rank throws; returns how many threads unwound.
int debugLoopbackAbort(int nranks, int failingRank, std::string* firstError);

} // namespace gs
