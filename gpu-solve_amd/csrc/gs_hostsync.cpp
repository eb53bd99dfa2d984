// gs_hostsync.cpp — HIP-free host logic of the exchange layer (see gs_hostsync.hpp).
#include "gs_hostsync.hpp"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#include <unistd.h>

#include "gs_params.hpp"

namespace gs {

double commTimeoutS(const char* env, double dflt)
{
    const char* e = std::getenv(env);
    if (!e || !*e) return dflt;
    const double v = std::strtod(e, nullptr);
    return v > 0 ? v : dflt;
}

std::string boundedWait(const std::function<int()>& poll, const std::function<std::string(int)>& errText,
                        double timeoutS, const char* what)
{
    const auto t0 = std::chrono::steady_clock::now();
    for (long spins = 0;; spins++) {
        const int st = poll();
        if (st == 0) return "";
        if (st != 1) return std::string(what) + ": " + errText(st);
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el > timeoutS) {
            char buf[160];
            std::snprintf(buf, sizeof buf, ": timed out after %.1f s (a peer is dead, deadlocked or far behind)", el);
            return std::string(what) + buf;
        }
        // spin briefly (a V-cycle's norm readback is ~1 ms away), then back off
        if (spins > 2000) std::this_thread::sleep_for(std::chrono::microseconds(spins > 20000 ? 1000 : 50));
    }
}

void publishUid(const std::string& path, const unsigned char* uid)
{
    const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) throw Error("cannot write the RCCL id file " + tmp);
    const bool ok = std::fwrite(uid, 1, 128, f) == 128;
    if (std::fclose(f) != 0 || !ok || std::rename(tmp.c_str(), path.c_str()) != 0) {
        std::remove(tmp.c_str());
        throw Error("cannot publish the RCCL id file " + path);
    }
}

void awaitUid(const std::string& path, double timeoutS, unsigned char* uid)
{
    const std::string err = boundedWait(
        [&]() -> int {
            FILE* f = std::fopen(path.c_str(), "rb");
            if (!f) return 1;
            const std::size_t n = std::fread(uid, 1, 128, f);
            std::fclose(f);
            return n == 128 ? 0 : 2;
        },
        [&](int) { return std::string("short RCCL id file ") + path; }, timeoutS, "waiting for rank 0's RCCL id");
    if (!err.empty()) throw Error(err + " (" + path + ")");
}

std::string uidPath()
{
    const char* e = std::getenv("GS_UID_FILE");
    if (e && *e) return e;
    const char* port = std::getenv("MASTER_PORT");
    std::string p = "/tmp/gpusolve-uid-" + std::to_string((long)getppid()) + "-" + (port && *port ? port : "0");
    // torchrun --max-restarts: the agent keeps its pid and port across attempts
    const char* run = std::getenv("TORCHELASTIC_RUN_ID");
    const char* restart = std::getenv("TORCHELASTIC_RESTART_COUNT");
    if (run && *run) {
        std::string r = run;
        for (char& c : r)
            if (c == '/' || c == '\0') c = '_';
        p += "-" + r;
    }
    if (restart && *restart) p += "-a" + std::string(restart);
    return p;
}

void LoopbackHub::barrier()
{
    std::unique_lock<std::mutex> lk(m_);
    if (aborted_) throw Error("loopback exchange aborted: " + why_);
    const int gen = gen_;
    if (++count_ == n_) {
        count_ = 0;
        gen_++;
        cv_.notify_all();
    } else {
        cv_.wait(lk, [&] { return gen != gen_ || aborted_; });
        if (gen == gen_) throw Error("loopback exchange aborted: " + why_);
    }
}

void LoopbackHub::abort(const std::string& why)
{
    std::lock_guard<std::mutex> lk(m_);
    if (!aborted_) why_ = why;
    aborted_ = true;
    cv_.notify_all();
}

std::string LoopbackHub::error()
{
    std::lock_guard<std::mutex> lk(m_);
    return aborted_ ? why_ : std::string();
}

int debugBoundedWait(int scenario, int k, double timeoutS, std::string* msg)
{
    int polls = 0;
    const std::string err = boundedWait(
        [&]() -> int {
            polls++;
            if (scenario == 0) return polls >= k ? 0 : 1;     // completes at poll k
            if (scenario == 1) return polls >= k ? 2 + 3 : 1; // asynchronous error (ncclInternalError = 3)
            return 1;                                          // never completes
        },
        [](int st) { return st == 5 ? std::string("internal error - please report this issue to the NCCL developers")
                                    : std::string("error ") + std::to_string(st); },
        timeoutS, "debug wait");
    if (msg) *msg = err;
    return err.empty() ? 0 : 1;
}

int debugLoopbackAbort(int nranks, int failingRank, std::string* firstError)
{
    // nranks threads meet at hub barriers; failingRank throws before its second barrier. Every
    // thread must unwind (no hang) and the first error must be the one reported.
    if (nranks < 1 || failingRank < 0 || failingRank >= nranks) return -1;
    LoopbackHub hub(nranks);
    std::vector<int> unwound(nranks, 0);
    auto body = [&](int r) {
        try {
            hub.barrier();
            if (r == failingRank) throw Error("rank " + std::to_string(r) + " failed");
            for (int i = 0; i < 3; i++) hub.barrier();
        } catch (const std::exception& e) {
            unwound[r] = 1;
            hub.abort(e.what());
        }
    };
    std::vector<std::thread> th;
    for (int r = 0; r < nranks; r++) th.emplace_back(body, r);
    for (auto& t : th) t.join();
    if (firstError) *firstError = hub.error();
    int n = 0;
    for (int u : unwound) n += u;
    return n; // == nranks when every rank unwound
}

} // namespace gs
