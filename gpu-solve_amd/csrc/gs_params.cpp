// gs_params.cpp — config reader and Timer (see gs_params.hpp).
#include "gs_params.hpp"

#include <fstream>
#include <iostream>
#include <sstream>
#include <sys/stat.h>

namespace gs {

namespace {

ConfigStatus parseStream(std::istream& in, GridParams& p)
{
    // field order: README.md:17-33 / src/main.cpp:34-82
    in >> p.maxiter >> p.tol >> p.gridDim[0] >> p.gridDim[1] >> p.gridDim[2];
    int mode = -1;
    in >> mode;
    if (mode < GridParams::LINEAR || mode > GridParams::NEWTON) return ConfigStatus::InvalidMode;
    p.mode = static_cast<GridParams::Mode>(mode);
    in >> p.preSmoothing >> p.postSmoothing >> p.omega >> p.gamma;
    for (auto& v : p.stencil.values) in >> v;
    int o = 0;
    for (auto& t : p.stencil.offsets) { in >> o; std::get<0>(t) = o; }
    for (auto& t : p.stencil.offsets) { in >> o; std::get<1>(t) = o; }
    for (auto& t : p.stencil.offsets) { in >> o; std::get<2>(t) = o; }
    for (std::size_t i = 0; i < 7; i++) {
        const int a = p.stencil.getXOffset(i), b = p.stencil.getYOffset(i), c = p.stencil.getZOffset(i);
        if (a < -1 || a > 1 || b < -1 || b > 1 || c < -1 || c > 1) return ConfigStatus::BadStencil;
    }
    p.h = 1.0 / (p.gridDim[1] + 1); // src/main.cpp:84
    return ConfigStatus::Ok;
}

} // namespace

ConfigStatus readConfig(const std::string& path, GridParams& p)
{
    struct stat st{};
    if (::stat(path.c_str(), &st) != 0 || !S_ISREG(st.st_mode)) return ConfigStatus::NotAFile;
    std::ifstream in(path);
    if (!in) return ConfigStatus::NotAFile;
    return parseStream(in, p);
}

ConfigStatus parseConfigText(const std::string& text, GridParams& p)
{
    std::istringstream in(text);
    return parseStream(in, p);
}

std::chrono::steady_clock::time_point Timer::t0_{};
std::map<std::string, Timer::Partial> Timer::parts_;

void Timer::start()
{
    parts_.clear();
    t0_ = std::chrono::steady_clock::now();
}

void Timer::stop()
{
    const auto ms =
        std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0_).count();
    std::cout << "Took " << ms << "ms";
    if (!parts_.empty()) {
        std::cout << ", ";
        for (const auto& kv : parts_) std::cout << kv.first << ": " << kv.second.ms << "ms (" << kv.second.count << "x) ";
    }
    std::cout << '\n';
}

void Timer::push(const std::string& name)
{
    Partial& t = parts_[name];
    t.last = std::chrono::steady_clock::now();
    t.count++;
}

void Timer::pop(const std::string& name)
{
    Partial& t = parts_.at(name);
    t.ms += std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t.last).count();
}

} // namespace gs
