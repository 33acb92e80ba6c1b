// ubench_ldsatomic.hip -- diagnostic (not product code): cost of the bin kernel's
// count atomics (ds_add_rtn_u32 on T per-tile counters, random tiles) with and
// without hash-like VALU work between them, at the bin kernel's occupancy (two
// 1024-thread blocks per CU, 72 KB of LDS each).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int VALU>
__global__ __launch_bounds__(1024, 8) void k(uint32_t *out, uint32_t T, uint32_t iters, uint32_t spread) {
    extern __shared__ uint32_t cnt[];
    for (uint32_t t = threadIdx.x; t < T; t += 1024) cnt[t] = 0;
    __syncthreads();
    uint32_t acc = 0;
    uint64_t x = (uint64_t)(blockIdx.x * 1024 + threadIdx.x) * 0x9E3779B97F4A7C15ull + 1;
    for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < VALU; ++j) x = (x ^ (x >> 29)) * 0xBF58476D1CE4E5B9ull;  // ~7 VALU each
        const uint32_t t = __umulhi((uint32_t)(x >> 32), T) * spread;
        acc += atomicAdd(&cnt[t], 4u);
    }
    if (acc == 0x12345u) out[0] = acc;
}

int main() {
    uint32_t *out;
    CK(hipMalloc(&out, 64));
    const size_t lds = 72 * 1024;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int valu : {0, 3}) {
        for (uint32_t T : {64u, 183u, 915u, 2048u}) {
            for (uint32_t spread : {1u, 33u}) {
                if (T * spread * 4 > lds) continue;
                auto kern = valu ? k<3> : k<0>;
                CK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                const uint32_t iters = 256, blocks = 256 * 2 * 8;
                hipLaunchKernelGGL(kern, dim3(blocks), dim3(1024), lds, 0, out, T, iters, spread);
                CK(hipDeviceSynchronize());
                float best = 1e9f;
                for (int r = 0; r < 3; ++r) {
                    CK(hipEventRecord(a));
                    hipLaunchKernelGGL(kern, dim3(blocks), dim3(1024), lds, 0, out, T, iters, spread);
                    CK(hipEventRecord(b));
                    CK(hipEventSynchronize(b));
                    float ms; CK(hipEventElapsedTime(&ms, a, b)); if (ms < best) best = ms;
                }
                const double wave_atomics_per_cu = (double)blocks * 16 * iters / 256;
                printf("valu=%d T=%4u spread=%2u: %.3f ms, %.2f cycles per wave-atomic per CU (2.4 GHz)\n",
                       valu, T, spread, best, best * 1e-3 * 2.4e9 / wave_atomics_per_cu);
            }
        }
    }
    return 0;
}
