// Compile-only probe (tools/glds_probe.sh): how hipcc (ROCm 7.2, gfx950) places s_waitcnt around
// __builtin_amdgcn_global_load_lds, the LDS-DMA form the round-2 verdict proposed for streaming f /
// newtonV into the NEWTON pairs. The loop has the pairs' structure at two plane steps of prefetch: four
// LDS slots (separate __shared__ objects so every slot index is static), step s issues the DMA of plane
// s+2 into slot (s+2)&3 and reads slot s&3, which was issued two steps earlier. The wait that read
// needs is vmcnt(<the DMAs issued after it>); the probe reports what the compiler emits.
#include <hip/hip_runtime.h>
typedef __attribute__((address_space(3))) void* lds_ptr;

__global__ __launch_bounds__(256) void k_glds_probe(const double* __restrict__ f, double* __restrict__ out, int n,
                                                    long ldz)
{
    __shared__ double2 s0[4][64], s1[4][64], s2[4][64], s3[4][64];
    const int w = threadIdx.y, l = threadIdx.x;
    const double* p = f + 2 * l + blockIdx.x * 512;
    auto dma = [&](auto& slot, int z) {
        __builtin_amdgcn_global_load_lds((const void*)(p + z * ldz), (lds_ptr)&slot[w][0], 16, 0, 0);
    };
    dma(s0, 0);
    dma(s1, 1);
    double acc = 0.0;
    for (int z = 0; z < n; z += 4) {
        dma(s2, z + 2);
        { const double2 a = s0[w][l]; acc += a.x * a.y; }
        dma(s3, z + 3);
        { const double2 a = s1[w][l]; acc += a.x * a.y; }
        dma(s0, z + 4);
        { const double2 a = s2[w][l]; acc += a.x * a.y; }
        dma(s1, z + 5);
        { const double2 a = s3[w][l]; acc += a.x * a.y; }
    }
    out[threadIdx.x + 64 * w + 256 * blockIdx.x] = acc;
}
