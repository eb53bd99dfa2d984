// gs_plan.cpp — Z-slab plane ownership of every level (pure host logic, no HIP / RCCL; built into the
// driver and, with -fsanitize=address,undefined, into the sanitizer harness: make -C oracle asan).
#include <cstdint>
#include <vector>

#include "gs_comm.hpp"

namespace gs {

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

} // namespace gs
