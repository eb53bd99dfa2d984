// gs_main.cpp — the GpuSolve-hip executable: drop-in for GpuSolve-cpu with the same CLI and stdout
// contract (src/main.cpp:15-114): `GpuSolve-hip <path/to/config.conf>`.
//
//   Using config file "<path>"
//   Solving linear|nonlinear|newton problem
//   Inital residual: R                       (sic, CpuSolver.cpp:17)
//   iter: i residual: R Took Tms             (CpuSolver.cpp:28 + Timer.cpp:17-26)
//   Inital newton residual: R / newton iter: i residual: R Took Tms   (NewtonSolver.cpp:16,27)
//
// Exit codes as the reference: 1 for a missing/non-file config or an invalid mode; a backend
// error prints "Exception: <what>" to stderr and exits 0 (the reference's GPU-backend behaviour,
// src/main.cpp:96-111). Added: stencil offsets outside {-1,0,1} (out-of-bounds reads in the
// reference) are rejected like an invalid mode. With GS_METRICS=1 one more line follows the solve:
// "[gs] mlups=... gbps=... pct_peak=... vcycle_ms=... cycles=... level_ms=..." (not matched by the
// reference harness's regex, runExperiments.py:46).
//
// Multi-GPU (added): started once per GPU by a launcher that sets WORLD_SIZE / RANK / LOCAL_RANK
// (`torchrun --nproc-per-node N --no-python GpuSolve-hip <conf>`), each process takes GPU LOCAL_RANK,
// rank 0's RCCL id reaches the others through a file (gs_comm.hpp uidPath), and the solve runs
// Z-slab partitioned; rank 0 prints the same stdout. GS_FORCE_RCCL=1 takes that path
// with one rank too (tests).
#include <cstdio>
#include <cstdlib>
#include <iomanip>
#include <iostream>
#include <memory>
#include <string>

#include <fcntl.h>
#include <unistd.h>

#include <hip/hip_runtime.h>

#include "gs_comm.hpp"
#include "gs_grid.hpp"
#include "gs_params.hpp"

namespace {
int envInt(const char* name, int dflt)
{
    const char* e = std::getenv(name);
    return e && *e ? std::atoi(e) : dflt;
}

// One process of a multi-GPU run: device, RCCL communicator, Z-slab grid, solve. Throws gs::Error.
void solveDistributed(const gs::GridParams& gridParams, int rank, int world)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) throw gs::Error("no HIP device");
    if (hipSetDevice(envInt("LOCAL_RANK", rank) % ndev) != hipSuccess) throw gs::Error("hipSetDevice failed");
    unsigned char uid[128] = {};
    const std::string path = gs::uidPath();
    if (rank == 0) {
        gs::rcclUniqueId(uid);
        gs::publishUid(path, uid);
    } else {
        gs::awaitUid(path, gs::commTimeoutS("GS_COMM_INIT_TIMEOUT_S", 300.0), uid);
    }
    // rank 0 removes the id file when it leaves (every rank's communicator exists by then, or the run failed)
    struct Cleanup {
        bool on;
        std::string p;
        ~Cleanup()
        {
            if (on) std::remove(p.c_str());
        }
    } cleanup{rank == 0, path};
    std::unique_ptr<gs::Comm> comm;
    {
        // RCCL prints a version banner to stdout at communicator creation: keep the reference's stdout
        // contract by sending fd 1 to /dev/null for that call only
        std::cout.flush();
        std::fflush(stdout);
        struct Quiet {
            int saved = dup(1);
            Quiet()
            {
                const int nul = open("/dev/null", O_WRONLY);
                if (saved >= 0 && nul >= 0) dup2(nul, 1);
                if (nul >= 0) close(nul);
            }
            ~Quiet()
            {
                std::fflush(stdout);
                if (saved >= 0) {
                    dup2(saved, 1);
                    close(saved);
                }
            }
        } quiet;
        comm = gs::makeRcclComm(rank, world, uid);
    }
    gs::HipGridData grid(gridParams, comm.get());
    // (the solvers print on rank 0 only; printProgress itself must be the same on every rank: it decides
    // whether the last closing norm, a collective, is computed)
    grid.printProgress = true;
    if (gridParams.mode == gs::GridParams::NEWTON) gs::NewtonSolver::solve(grid);
    else gs::HipSolver::solve(grid);
    if (grid.clock.on && rank == 0) std::cout << gs::metricsLine(grid) << '\n';
}
} // namespace

int main(int argc, char* argv[])
{
    if (argc < 2) {
        std::cerr << "Missing config file. Usage program.exe path/to/config.conf\n";
        return 1;
    }
    const std::string path = argv[1];
    gs::GridParams gridParams;
    // read the mode first so the "Using"/"Solving" lines come out in the reference's order
    const gs::ConfigStatus st = gs::readConfig(path, gridParams);
    if (st == gs::ConfigStatus::NotAFile) {
        std::cerr << std::quoted(path) << " does not exist or is not a file\n";
        return 1;
    }
    const int world = envInt("WORLD_SIZE", 1), rank = envInt("RANK", 0);
    const bool distributed = world > 1 || envInt("GS_FORCE_RCCL", 0) != 0;
    if (distributed) {
        // RCCL's p2p channels per peer fill the communicator's CTA budget (gs_comm.hpp): RCCL reads the
        // variable once per process, so it is set here, before HIP, RCCL or any thread starts (an explicit
        // value in the environment wins)
        if (const int cpp = gs::rcclChannelsPerPeerHint(); cpp > 0)
            setenv("NCCL_NCHANNELS_PER_PEER", std::to_string(cpp).c_str(), 0);
    }
    if (rank == 0) std::cout << "Using config file " << std::quoted(path) << '\n';
    if (st == gs::ConfigStatus::InvalidMode) {
        std::cerr << "Invalid mode\n";
        return 1;
    }
    if (rank == 0) {
        if (gridParams.mode == gs::GridParams::LINEAR) std::cout << "Solving linear problem\n";
        else if (gridParams.mode == gs::GridParams::NONLINEAR) std::cout << "Solving nonlinear problem\n";
        else std::cout << "Solving newton problem\n";
    }
    if (st == gs::ConfigStatus::BadStencil) {
        std::cerr << "Invalid stencil offset (must be -1, 0 or 1)\n";
        return 1;
    }

    if (distributed) {
        if (rank < 0 || rank >= world) {
            std::cerr << "Exception: RANK " << rank << " outside WORLD_SIZE " << world << '\n';
            return 0;
        }
        try {
            solveDistributed(gridParams, rank, world);
            if (argc > 2 && rank == 0) std::cerr << "(the solution dump is written by single-GPU runs only)\n";
        } catch (std::exception& e) {
            std::cerr << "Exception: " << e.what() << '\n';
        }
        return 0;
    }

    try {
        gs::HipGridData grid(gridParams);
        if (gridParams.mode == gs::GridParams::NEWTON) gs::NewtonSolver::solve(grid);
        else gs::HipSolver::solve(grid);
        if (grid.clock.on) std::cout << gs::metricsLine(grid) << '\n'; // GS_METRICS=1 (added, optional)
        if (argc > 2) gs::dumpField(grid, 0, argv[2]); // Vector3::dump of the solution (added, optional)
    } catch (std::exception& e) {
        std::cerr << "Exception: " << e.what() << '\n';
    }
    return 0;
}
