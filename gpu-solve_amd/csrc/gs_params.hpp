// gs_params.hpp — problem description, config-file reader and progress timer of GpuSolve-hip.
//
// Mirrors the reference's interface so GpuSolve-hip is a drop-in next to GpuSolve-cpu:
//   GridParams / Stencil      src/gridParams.h:7-47   (same field names and meaning)
//   14-line config file        src/main.cpp:32-85, README.md:17-33
//   Timer ("Took Nms")         src/Timer.{h,cpp}
#pragma once
#include <array>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <tuple>

namespace gs {

struct Stencil {
    std::array<double, 7> values{};
    std::array<std::tuple<int, int, int>, 7> offsets{};
    int getXOffset(std::size_t i) const { return std::get<0>(offsets[i]); }
    int getYOffset(std::size_t i) const { return std::get<1>(offsets[i]); }
    int getZOffset(std::size_t i) const { return std::get<2>(offsets[i]); }
};

struct GridParams {
    enum Mode { LINEAR, NONLINEAR, NEWTON };

    std::size_t maxiter = 0;
    double tol = 0.0;
    double omega = 0.0; // relaxation coefficient
    double gamma = 0.0; // non-linear weight
    double h = 0.0;
    std::array<std::size_t, 3> gridDim{};
    std::size_t preSmoothing = 0;
    std::size_t postSmoothing = 0;
    Stencil stencil{};
    Mode mode = LINEAR;

    // rank 0 prints the solve's progress; on a Z-slab grid the flag must be the same on every rank (it also
    // decides whether a solve's last, otherwise unread closing norm — a collective — is computed)
    bool printProgress = true;
};

// Error raised by the HIP backend (the reference prints "Exception: <what>", src/main.cpp:107-109).
struct Error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

enum class ConfigStatus { Ok, NotAFile, InvalidMode, BadStencil };

// Reads the 14 whitespace-separated fields in the reference's order. Like the reference, missing
// trailing fields leave defaults; unlike it, stencil offsets outside {-1,0,1} (which would index
// outside the padded grid) are rejected with BadStencil.
ConfigStatus readConfig(const std::string& path, GridParams& p);

// Same reader on an in-memory config text (used by the C ABI).
ConfigStatus parseConfigText(const std::string& text, GridParams& p);

class Timer {
public:
    static void start();
    static void stop(); // prints "Took Nms[, name: Nms (kx) ...]\n"
    static void push(const std::string& name);
    static void pop(const std::string& name);

private:
    struct Partial {
        uint64_t ms = 0, count = 0;
        std::chrono::steady_clock::time_point last{};
    };
    static std::chrono::steady_clock::time_point t0_;
    static std::map<std::string, Partial> parts_;
};

} // namespace gs
