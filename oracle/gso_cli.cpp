// gso_cli.cpp — CLI over the CPU oracle (TEST INFRASTRUCTURE / cpu_baseline only).
//   gso_cli <config>                       reference-format run (src/main.cpp:15-114 stdout contract)
//   gso_cli --digits17 <config>            same, residuals at 17 significant digits
//   gso_cli time_jacobi X Y Z mode sweeps  JSON: Jacobi MLUPS on level 0
//   gso_cli time_vcycle X Y Z mode cycles  JSON: ms per 2+2 V-cycle
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>

extern "C" {
typedef struct { double s[7]; int ox[7], oy[7], oz[7]; } gso_stencil;
void* gso_grid_create(const gso_stencil*, const int64_t*, int, int64_t, double, double, double, int64_t, int64_t);
void gso_grid_destroy(void*);
int gso_grid_solve(void*, int, double*, int);
int gso_num_threads(void);
double gso_time_jacobi(const gso_stencil*, const int64_t*, int, int);
double gso_time_vcycle(const gso_stencil*, const int64_t*, int, int, double*);
}

static gso_stencil std7()
{
    gso_stencil S{{6, -1, -1, -1, -1, -1, -1}, {0, 1, -1, 0, 0, 0, 0}, {0, 0, 0, 1, -1, 0, 0}, {0, 0, 0, 0, 0, 1, -1}};
    return S;
}

int main(int argc, char** argv)
{
    if (argc >= 7 && (!std::strcmp(argv[1], "time_jacobi") || !std::strcmp(argv[1], "time_vcycle"))) {
        gso_stencil S = std7();
        int64_t d[3] = {std::atoll(argv[2]), std::atoll(argv[3]), std::atoll(argv[4])};
        int mode = std::atoi(argv[5]), k = std::atoi(argv[6]);
        if (!std::strcmp(argv[1], "time_jacobi")) {
            double s = gso_time_jacobi(&S, d, mode, k);
            std::printf("{\"sweeps\": %d, \"seconds\": %.6f, \"mlups\": %.3f, \"threads\": %d}\n", k, s,
                        double(d[0]) * d[1] * d[2] * k / s / 1e6, gso_num_threads());
        } else {
            double r = 0, s = gso_time_vcycle(&S, d, mode, k, &r);
            std::printf("{\"cycles\": %d, \"ms_per_cycle\": %.3f, \"residual\": %.17g, \"threads\": %d}\n", k, s * 1e3, r,
                        gso_num_threads());
        }
        return 0;
    }
    int ai = 1;
    bool d17 = false;
    if (argc > 2 && !std::strcmp(argv[1], "--digits17")) { d17 = true; ai = 2; }
    if (ai >= argc) { std::fprintf(stderr, "usage: gso_cli [--digits17] <config>\n"); return 1; }
    std::ifstream in(argv[ai]);
    if (!in) { std::fprintf(stderr, "\"%s\" does not exist or is not a file\n", argv[ai]); return 1; }
    int64_t maxiter, d[3], pre, post;
    double tol, omega, gamma;
    int mode;
    gso_stencil S;
    in >> maxiter >> tol >> d[0] >> d[1] >> d[2] >> mode >> pre >> post >> omega >> gamma;
    for (int i = 0; i < 7; i++) in >> S.s[i];
    for (int i = 0; i < 7; i++) in >> S.ox[i];
    for (int i = 0; i < 7; i++) in >> S.oy[i];
    for (int i = 0; i < 7; i++) in >> S.oz[i];
    void* g = gso_grid_create(&S, d, mode, maxiter, tol, omega, gamma, pre, post);
    gso_grid_solve(g, d17 ? 2 : 1, nullptr, 0);
    gso_grid_destroy(g);
    return 0;
}
