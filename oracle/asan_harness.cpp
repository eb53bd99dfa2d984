// asan_harness.cpp — TEST INFRASTRUCTURE: the host-only code under -fsanitize=address,undefined
// (SURVEY.md §5 "race detection / sanitizers"; built by `make -C oracle asan`, run by
// tests/test_sanitizers.py). Exercises
//   * the CPU oracle restatement (oracle/gs_oracle.cpp): whole solves in all three modes on odd, even,
//     non-cubic and degenerate grids, and every per-operator entry point;
//   * the product's config reader (gpu-solve_amd/csrc/gs_params.cpp: valid, truncated, garbage, bad
//     mode / stencil texts — the reference reads these fields unvalidated, src/main.cpp:32-85);
//   * the product's Z-slab ownership plan (gpu-solve_amd/csrc/gs_plan.cpp) over many grids and rank
//     counts, checking its invariants;
//   * the exchange layer's HIP-free host logic (gpu-solve_amd/csrc/gs_hostsync.cpp): the bounded wait
//     that settles every RCCL call (completion, error, timeout), the rank-0 id file hand-off (publish /
//     await / a stale file of an earlier torchrun attempt), and the loopback hub's barrier/abort across
//     rank threads.
// Built twice: `asan` (address + undefined, everything) and `tsan` (-DGS_HOSTSYNC_ONLY, thread
// sanitizer over the host-sync section alone: the OpenMP oracle is not TSan-instrumented).
// Any sanitizer report aborts (-fno-sanitize-recover=all); an invariant failure exits 1.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <unistd.h>

#include "gs_comm.hpp"
#include "gs_hostsync.hpp"
#include "gs_params.hpp"

#ifndef GS_HOSTSYNC_ONLY
extern "C" {
typedef struct { double s[7]; int ox[7], oy[7], oz[7]; } gso_stencil;
void* gso_grid_create(const gso_stencil*, const int64_t*, int, int64_t, double, double, double, int64_t, int64_t);
void gso_grid_destroy(void*);
int gso_grid_solve(void*, int, double*, int);
double gso_residual(const gso_stencil*, const int64_t n[3], double h, int mode, double gamma, const double* v,
                    const double* f, const double* w, double* r);
void gso_jacobi(const gso_stencil*, const int64_t n[3], double h, int mode, double omega, double gamma, int sweeps,
                double* v, const double* f, const double* w, double* r_scratch);
double gso_newton_F(const gso_stencil*, const int64_t n[3], double h, double gamma, const double* w, const double* F,
                    double* f);
void gso_apply_op(const gso_stencil*, const int64_t n[3], double h, double gamma, const double* u, double* out);
void gso_restrict(const double* fine, const int64_t fn[3], double* coarse, const int64_t cn[3]);
void gso_interpolate(const double* coarse, const int64_t cn[3], double* e, const int64_t fn[3]);
void gso_rhs(const int64_t n[3], double h, int mode, double gamma, double* f);
}
#endif

namespace {

int failures = 0;
#define CHECK(c)                                                                                                       \
    do {                                                                                                               \
        if (!(c)) {                                                                                                    \
            std::fprintf(stderr, "CHECK failed: %s (%s:%d)\n", #c, __FILE__, __LINE__);                                \
            failures++;                                                                                                \
        }                                                                                                              \
    } while (0)

#ifndef GS_HOSTSYNC_ONLY
const gso_stencil S7{{6, -1, -1, -1, -1, -1, -1}, {0, 1, -1, 0, 0, 0, 0}, {0, 0, 0, 1, -1, 0, 0}, {0, 0, 0, 0, 0, 1, -1}};

std::size_t padded(const int64_t n[3]) { return (std::size_t)((n[0] + 2) * (n[1] + 2) * (n[2] + 2)); }

void solves()
{
    const int64_t dims[][3] = {{1, 1, 1}, {2, 3, 1}, {7, 7, 7}, {8, 8, 8}, {15, 9, 12}, {16, 17, 5}, {31, 31, 31}};
    for (const auto& d : dims)
        for (int mode = 0; mode < 3; mode++)
            for (int pre = 0; pre <= 3; pre += 3) {
                void* g = gso_grid_create(&S7, d, mode, mode == 2 ? 2 : 3, 0.0, 0.8, 1.0, pre, 2);
                double hist[16] = {};
                const int n = gso_grid_solve(g, 0, hist, 16);
                CHECK(n >= 1 && n <= 16);
                gso_grid_destroy(g);
            }
}

void operators()
{
    const int64_t n[3] = {13, 6, 10}, c[3] = {6, 3, 5};
    std::vector<double> v(padded(n)), f(padded(n)), w(padded(n)), r(padded(n)), e(padded(n)), cv(padded(c));
    unsigned s = 1;
    auto rnd = [&] { s = s * 1103515245u + 12345u; return (double)(s >> 8) / (1u << 24) - 0.5; };
    for (int64_t x = 1; x <= n[0]; x++)
        for (int64_t y = 1; y <= n[1]; y++)
            for (int64_t z = 1; z <= n[2]; z++) {
                const std::size_t i = (std::size_t)(z + (n[2] + 2) * (y + (n[1] + 2) * x));
                v[i] = rnd();
                w[i] = rnd();
            }
    const double h = 1.0 / (n[1] + 1);
    for (int mode = 0; mode < 3; mode++) {
        gso_rhs(n, h, mode, 1.0, f.data());
        const double nr = gso_residual(&S7, n, h, mode, 1.0, v.data(), f.data(), w.data(), r.data());
        CHECK(nr > 0);
        gso_jacobi(&S7, n, h, mode, 0.8, 1.0, 2, v.data(), f.data(), w.data(), r.data());
    }
    CHECK(gso_newton_F(&S7, n, h, 1.0, w.data(), f.data(), e.data()) > 0);
    gso_apply_op(&S7, n, h, 1.0, v.data(), r.data());
    gso_restrict(r.data(), n, cv.data(), c);
    gso_interpolate(cv.data(), c, e.data(), n);
}

void configs()
{
    const std::string stencil = "6 -1 -1 -1 -1 -1 -1\n0 1 -1 0 0 0 0\n0 0 0 1 -1 0 0\n0 0 0 0 0 1 -1\n";
    struct Case {
        std::string text;
        gs::ConfigStatus want;
    } cases[] = {
        {"10\n1e-5\n127\n127\n127\n2\n3\n3\n0.8\n1.0\n" + stencil, gs::ConfigStatus::Ok},
        {"10\n0\n7\n7\n7\n5\n2\n2\n0.8\n1.0\n" + stencil, gs::ConfigStatus::InvalidMode},
        {"10\n0\n7\n7\n7\n-1\n", gs::ConfigStatus::InvalidMode},
        {"10\n0\n7\n7\n7\n0\n2\n2\n0.8\n1.0\n6 -1 -1 -1 -1 -1 -1\n0 2 -1 0 0 0 0\n0 0 0 1 -1 0 0\n0 0 0 0 0 1 -1\n",
         gs::ConfigStatus::BadStencil},
        {"", gs::ConfigStatus::InvalidMode},
        {"garbage \x01\x02 text", gs::ConfigStatus::InvalidMode},
        {"10\n0\n7\n7\n7\n0\n", gs::ConfigStatus::Ok}, // truncated after the mode: defaults stay
    };
    for (const auto& c : cases) {
        gs::GridParams p;
        CHECK(gs::parseConfigText(c.text, p) == c.want);
    }
    gs::GridParams p;
    CHECK(gs::readConfig("/nonexistent/path.conf", p) == gs::ConfigStatus::NotAFile);
    CHECK(gs::readConfig("/", p) == gs::ConfigStatus::NotAFile);
}

void plans()
{
    for (int64_t nz : {1, 2, 3, 7, 9, 16, 31, 63, 64, 127, 128, 1024})
        for (int nranks : {1, 2, 3, 4, 7, 8, 16})
            for (int64_t minPts : {(int64_t)0, (int64_t)4096, (int64_t)32768}) {
                std::vector<int64_t> nzs, pts;
                for (int64_t z = nz, xy = 64; z >= 1; z /= 2, xy /= 2) {
                    nzs.push_back(z);
                    pts.push_back(z * (xy > 0 ? xy : 1) * (xy > 0 ? xy : 1));
                }
                const gs::SlabPlan pl = gs::planZSlabs(nzs, pts, nranks, minPts);
                CHECK(pl.distributed.size() == nzs.size());
                CHECK(!pl.distributed.back());
                for (std::size_t l = 0; l < nzs.size(); l++) {
                    if (l && !pl.distributed[l - 1]) CHECK(!pl.distributed[l]);
                    if (!(l == 0 || pl.distributed[l - 1])) continue;
                    int64_t covered = 0;
                    for (int r = 0; r < nranks; r++)
                        if (pl.hi[l][r] >= pl.lo[l][r]) covered += pl.hi[l][r] - pl.lo[l][r] + 1;
                    CHECK(covered == nzs[l]);
                }
            }
}

#endif // GS_HOSTSYNC_ONLY

void hostsync()
{
    // bounded wait: completes at poll k, an asynchronous error at poll k, a timeout
    std::string msg;
    CHECK(gs::debugBoundedWait(0, 5, 10.0, &msg) == 0 && msg.empty());
    CHECK(gs::debugBoundedWait(1, 3, 10.0, &msg) == 1 && msg.find("internal error") != std::string::npos);
    CHECK(gs::debugBoundedWait(2, 0, 0.05, &msg) == 1 && msg.find("timed out") != std::string::npos);
    // loopback hub: every rank thread unwinds when one fails, whichever it is
    for (int n : {1, 2, 3, 8})
        for (int f = 0; f < n; f++) {
            std::string first;
            CHECK(gs::debugLoopbackAbort(n, f, &first) == n);
            CHECK(first == "rank " + std::to_string(f) + " failed");
        }
    // id hand-off: publish -> await round trip; a stale file of attempt 0 is not the path of attempt 1
    char dir[] = "/tmp/gs_hostsync_XXXXXX";
    CHECK(mkdtemp(dir) != nullptr);
    const std::string path = std::string(dir) + "/uid";
    unsigned char a[128], b[128] = {};
    for (int i = 0; i < 128; i++) a[i] = (unsigned char)(i * 7 + 1);
    gs::publishUid(path, a);
    gs::awaitUid(path, 5.0, b);
    CHECK(std::memcmp(a, b, 128) == 0);
    bool threw = false;
    try {
        gs::awaitUid(path + ".missing", 0.05, b);
    } catch (const gs::Error&) {
        threw = true;
    }
    CHECK(threw);
    unsetenv("GS_UID_FILE");
    setenv("MASTER_PORT", "29500", 1);
    setenv("TORCHELASTIC_RUN_ID", "run/1", 1);
    setenv("TORCHELASTIC_RESTART_COUNT", "0", 1);
    const std::string p0 = gs::uidPath();
    setenv("TORCHELASTIC_RESTART_COUNT", "1", 1);
    const std::string p1 = gs::uidPath();
    CHECK(p0 != p1 && p0.rfind('/') == 4); // one file under /tmp, the run id's '/' replaced
    unsetenv("TORCHELASTIC_RUN_ID");
    unsetenv("TORCHELASTIC_RESTART_COUNT");
    std::remove(path.c_str());
    rmdir(dir);
}

} // namespace

int main()
{
#ifndef GS_HOSTSYNC_ONLY
    solves();
    operators();
    configs();
    plans();
#endif
    hostsync();
    if (failures) {
        std::fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    std::printf("asan harness ok\n");
    return 0;
}
