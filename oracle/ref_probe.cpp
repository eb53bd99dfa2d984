// ref_probe.cpp — TEST INFRASTRUCTURE ONLY (oracle pinning; never shipped, never measured as product).
//
// A probe `main` of our own that links the reference's CPU backend *from where it lies*
// (/root/reference/src/cpu/*.cpp + Timer.cpp, compiled by oracle/Makefile into oracle/_ref/).
// No reference source is copied into this repository. It exposes the reference's own
// operators so we can:
//   * print residual histories at 17 significant digits (the reference prints 6),
//   * dump per-operator outputs on seeded random fields (golden fixtures, tests/golden/),
//   * time CpuSolver::jacobi / vcycle for the cpu_baseline leg of bench.py (kind "reference").
//
// Reference entry points exercised (file:line in /root/reference):
//   CpuSolver::solve          src/cpu/CpuSolver.cpp:12-43
//   CpuSolver::compResidual   src/cpu/CpuSolver.cpp:45-83
//   CpuSolver::vcycle         src/cpu/CpuSolver.cpp:85-139
//   CpuSolver::jacobi         src/cpu/CpuSolver.cpp:141-180
//   CpuSolver::applyStencil   src/cpu/CpuSolver.cpp:182-208
//   CpuSolver::restrict       src/cpu/CpuSolver.cpp:211-238
//   CpuSolver::interpolate    src/cpu/CpuSolver.cpp:240-290
//   NewtonSolver::solve/compF src/cpu/NewtonSolver.cpp:10-81
//   CpuGridData ctor (levels, h, RHS) src/cpu/CpuGridData.cpp:15-79
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <random>
#include <string>
#include <tuple>
#include <vector>
#include <omp.h>

// Reach the reference's private statics (jacobi, compResidual, ...) and Vector3::values.
#define private public
#include "cpu/CpuGridData.h"
#include "cpu/CpuSolver.h"
#include "cpu/NewtonSolver.h"
#undef private

namespace {

GridParams make_params(std::size_t X, std::size_t Y, std::size_t Z, int mode, std::size_t pre,
                       std::size_t post, double omega, double gamma, std::size_t maxiter, double tol)
{
    GridParams p;
    p.maxiter = maxiter;
    p.tol = tol;
    p.gridDim = {X, Y, Z};
    p.mode = static_cast<GridParams::Mode>(mode);
    p.preSmoothing = pre;
    p.postSmoothing = post;
    p.omega = omega;
    p.gamma = gamma;
    // standard 7-point Laplacian, config order of examples/data-2nd_order.conf:11-14
    const double vals[7] = {6, -1, -1, -1, -1, -1, -1};
    const int ox[7] = {0, 1, -1, 0, 0, 0, 0};
    const int oy[7] = {0, 0, 0, 1, -1, 0, 0};
    const int oz[7] = {0, 0, 0, 0, 0, 1, -1};
    for (int i = 0; i < 7; i++) {
        p.stencil.values[i] = vals[i];
        p.stencil.offsets[i] = std::make_tuple(ox[i], oy[i], oz[i]);
    }
    p.h = 1.0 / (Y + 1);
    return p;
}

// Read a 14-field config file (README.md:17-33 order) into GridParams.
bool read_config(const char* path, GridParams& p)
{
    std::ifstream in(path);
    if (!in) return false;
    int mode = 0;
    in >> p.maxiter >> p.tol >> p.gridDim[0] >> p.gridDim[1] >> p.gridDim[2] >> mode >> p.preSmoothing >>
        p.postSmoothing >> p.omega >> p.gamma;
    p.mode = static_cast<GridParams::Mode>(mode);
    for (int i = 0; i < 7; i++) in >> p.stencil.values[i];
    int o;
    for (int i = 0; i < 7; i++) { in >> o; std::get<0>(p.stencil.offsets[i]) = o; }
    for (int i = 0; i < 7; i++) { in >> o; std::get<1>(p.stencil.offsets[i]) = o; }
    for (int i = 0; i < 7; i++) { in >> o; std::get<2>(p.stencil.offsets[i]) = o; }
    p.h = 1.0 / (p.gridDim[1] + 1);
    return static_cast<bool>(in);
}

// Seeded U(-1,1) on the interior, zero on the padding (the invariant every solver path keeps).
void fill_random(Vector3& v, std::mt19937_64& rng)
{
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    for (std::size_t x = 0; x < v.getXdim(); x++)
        for (std::size_t y = 0; y < v.getYdim(); y++)
            for (std::size_t z = 0; z < v.getZdim(); z++) {
                bool interior = x > 0 && y > 0 && z > 0 && x + 1 < v.getXdim() && y + 1 < v.getYdim() &&
                                z + 1 < v.getZdim();
                v.values[z + y * v.getZdim() + x * v.getZdim() * v.getYdim()] = interior ? U(rng) : 0.0;
            }
}

void dump(const Vector3& v, const std::string& path)
{
    std::FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) { std::perror(path.c_str()); std::exit(2); }
    std::fwrite(v.values.data(), sizeof(double), v.values.size(), f);
    std::fclose(f);
}

int usage()
{
    std::cerr << "usage:\n"
                 "  ref_probe solve <config>                      (17-digit residual history)\n"
                 "  ref_probe solve_dump <config> out.txt out.bin (Vector3::dump of level-0 v after the solve)\n"
                 "  ref_probe levels X Y Z\n"
                 "  ref_probe rhs X Y Z mode gamma out.bin\n"
                 "  ref_probe op <name> X Y Z mode level seed outdir [omega gamma k]\n"
                 "  ref_probe time_jacobi X Y Z mode sweeps       (MLUPS of CpuSolver::jacobi, level 0)\n"
                 "  ref_probe time_vcycle X Y Z mode cycles       (ms per CpuSolver::vcycle, 2+2)\n";
    return 1;
}

} // namespace

int main(int argc, char** argv)
{
    if (argc < 2) return usage();
    const std::string cmd = argv[1];
    std::cout << std::setprecision(17);

    if (cmd == "solve" && argc >= 3) {
        GridParams p;
        if (!read_config(argv[2], p)) { std::cerr << "bad config\n"; return 1; }
        CpuGridData g(p);
        if (p.mode == GridParams::NEWTON) NewtonSolver::solve(g);
        else CpuSolver::solve(g);
        return 0;
    }
    if (cmd == "solve_dump" && argc >= 5) {
        // solve quietly, then the reference's own Vector3::dump of level-0 v (text) + raw doubles
        GridParams p;
        if (!read_config(argv[2], p)) { std::cerr << "bad config\n"; return 1; }
        CpuGridData g(p);
        std::streambuf* old = std::cout.rdbuf(nullptr);
        if (p.mode == GridParams::NEWTON) NewtonSolver::solve(g);
        else CpuSolver::solve(g);
        std::cout.rdbuf(old);
        g.getLevel(0).v.dump(argv[3]);
        dump(g.getLevel(0).v, argv[4]);
        return 0;
    }
    if (cmd == "levels" && argc >= 5) {
        GridParams p = make_params(std::atol(argv[2]), std::atol(argv[3]), std::atol(argv[4]), 0, 1, 1, 0.8, 1.0, 1, 0.0);
        CpuGridData g(p);
        for (std::size_t l = 0; l < g.numLevels(); l++) {
            auto& L = g.getLevel(l);
            std::cout << l << ' ' << L.levelDim[0] << ' ' << L.levelDim[1] << ' ' << L.levelDim[2] << ' ' << L.h
                      << ' ' << (L.e.flatSize() > 0 ? 1 : 0) << '\n';
        }
        return 0;
    }
    if (cmd == "rhs" && argc >= 8) {
        GridParams p = make_params(std::atol(argv[2]), std::atol(argv[3]), std::atol(argv[4]), std::atoi(argv[5]), 1, 1,
                                   0.8, std::atof(argv[6]), 1, 0.0);
        CpuGridData g(p);
        dump(g.getLevel(0).f, argv[7]);
        return 0;
    }
    if (cmd == "op" && argc >= 10) {
        const std::string name = argv[2];
        const std::size_t X = std::atol(argv[3]), Y = std::atol(argv[4]), Z = std::atol(argv[5]);
        const int mode = std::atoi(argv[6]);
        const std::size_t lvl = std::atol(argv[7]);
        std::mt19937_64 rng(std::strtoull(argv[8], nullptr, 10));
        const std::string out = argv[9];
        const double omega = argc > 10 ? std::atof(argv[10]) : 0.8;
        const double gamma = argc > 11 ? std::atof(argv[11]) : 1.0;
        const std::size_t k = argc > 12 ? std::atol(argv[12]) : 1;
        GridParams p = make_params(X, Y, Z, mode, 2, 2, omega, gamma, 1, 0.0);
        CpuGridData g(p);
        auto& L = g.getLevel(lvl);
        if (name == "residual") {
            fill_random(L.v, rng); fill_random(L.f, rng); fill_random(L.newtonV, rng);
            dump(L.v, out + "/v.bin"); dump(L.f, out + "/f.bin"); dump(L.newtonV, out + "/newtonV.bin");
            double n = CpuSolver::compResidual(g, lvl);
            dump(L.r, out + "/r.bin");
            std::cout << "norm " << n << '\n';
        } else if (name == "jacobi") {
            fill_random(L.v, rng); fill_random(L.f, rng); fill_random(L.newtonV, rng);
            dump(L.v, out + "/v.bin"); dump(L.f, out + "/f.bin"); dump(L.newtonV, out + "/newtonV.bin");
            CpuSolver::jacobi(g, lvl, k);
            dump(L.v, out + "/v_out.bin");
        } else if (name == "restrict") {
            fill_random(L.r, rng);
            dump(L.r, out + "/fine.bin");
            CpuSolver::restrict(L.r, g.getLevel(lvl + 1).f);
            dump(g.getLevel(lvl + 1).f, out + "/coarse.bin");
        } else if (name == "interpolate") {
            auto& C = g.getLevel(lvl + 1);
            fill_random(C.v, rng);
            dump(C.v, out + "/coarse.bin");
            CpuSolver::interpolate(g, lvl);
            dump(L.e, out + "/e.bin");
        } else if (name == "applyStencil") {
            fill_random(L.restV, rng);
            dump(L.restV, out + "/u.bin");
            CpuSolver::applyStencil(g, lvl, L.restV);
            dump(L.r, out + "/r.bin");
        } else if (name == "compF") {
            auto& L0 = g.getLevel(0);
            fill_random(L0.newtonV, rng);
            g.newtonF = Vector3(X + 2, Y + 2, Z + 2);
            fill_random(g.newtonF, rng);
            dump(L0.newtonV, out + "/newtonV.bin"); dump(g.newtonF, out + "/newtonF.bin");
            double n = NewtonSolver::compF(g);
            dump(L0.f, out + "/f.bin");
            std::cout << "norm " << n << '\n';
        } else if (name == "vcycle") {
            // one V-cycle from a random level-0 iterate (analytic RHS kept); Newton: random newtonV on all levels
            fill_random(g.getLevel(0).v, rng);
            for (std::size_t l = 0; l < g.numLevels(); l++) fill_random(g.getLevel(l).newtonV, rng);
            for (std::size_t l = 0; l < g.numLevels(); l++) dump(g.getLevel(l).newtonV, out + "/newtonV" + std::to_string(l) + ".bin");
            dump(g.getLevel(0).v, out + "/v.bin");
            dump(g.getLevel(0).f, out + "/f.bin");
            double n = CpuSolver::vcycle(g);
            dump(g.getLevel(0).v, out + "/v_out.bin");
            std::cout << "norm " << n << '\n';
        } else {
            return usage();
        }
        return 0;
    }
    if (cmd == "time_jacobi" && argc >= 7) {
        const std::size_t X = std::atol(argv[2]), Y = std::atol(argv[3]), Z = std::atol(argv[4]);
        GridParams p = make_params(X, Y, Z, std::atoi(argv[5]), 2, 2, 0.8, 1.0, 1, 0.0);
        const int sweeps = std::atoi(argv[6]);
        CpuGridData g(p);
        CpuSolver::jacobi(g, 0, 1); // first touch
        auto t0 = std::chrono::steady_clock::now();
        CpuSolver::jacobi(g, 0, sweeps);
        auto t1 = std::chrono::steady_clock::now();
        double s = std::chrono::duration<double>(t1 - t0).count();
        double lups = double(X) * Y * Z * sweeps;
        std::cout << "{\"sweeps\": " << sweeps << ", \"seconds\": " << s << ", \"mlups\": " << lups / s / 1e6
                  << ", \"threads\": " << omp_get_max_threads() << "}\n";
        return 0;
    }
    if (cmd == "time_vcycle" && argc >= 7) {
        const std::size_t X = std::atol(argv[2]), Y = std::atol(argv[3]), Z = std::atol(argv[4]);
        GridParams p = make_params(X, Y, Z, std::atoi(argv[5]), 2, 2, 0.8, 1.0, 1, 0.0);
        const int cycles = std::atoi(argv[6]);
        CpuGridData g(p);
        CpuSolver::vcycle(g); // first touch
        auto t0 = std::chrono::steady_clock::now();
        double r = 0;
        for (int c = 0; c < cycles; c++) r = CpuSolver::vcycle(g);
        auto t1 = std::chrono::steady_clock::now();
        double s = std::chrono::duration<double>(t1 - t0).count();
        std::cout << "{\"cycles\": " << cycles << ", \"seconds\": " << s << ", \"ms_per_cycle\": " << 1e3 * s / cycles
                  << ", \"residual\": " << r << ", \"threads\": " << omp_get_max_threads() << "}\n";
        return 0;
    }
    return usage();
}
