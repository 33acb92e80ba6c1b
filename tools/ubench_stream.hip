// Attainable HBM bandwidth on this box ("also report vs a measured
// streaming-read kernel"): a 16-byte-per-lane grid-stride read, write and copy over
// 4 GiB buffers, best of 10 launches each.  Build:
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_stream.hip -o tools/ubench_stream
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);         \
            std::exit(1);                                                                \
        }                                                                                \
    } while (0)

__global__ __launch_bounds__(256) void read_kernel(const v4u *__restrict__ src, size_t n,
                                                   uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const v4u v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;  // keeps the loads alive
}

__global__ __launch_bounds__(256) void write_kernel(v4u *__restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        dst[i] = v4u{(uint32_t)i, 0u, 0u, 0u};
}

__global__ __launch_bounds__(256) void copy_kernel(const v4u *__restrict__ src, v4u *__restrict__ dst,
                                                   size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        dst[i] = src[i];
}

int main() {
    const size_t bytes = 4ull << 30, n = bytes / 16;
    v4u *a, *b;
    uint32_t *sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 1 << 20));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int grid : {1024, 2048, 4096, 8192}) {
        float best[3] = {1e9f, 1e9f, 1e9f};
        for (int rep = 0; rep < 11; ++rep) {
            for (int w = 0; w < 3; ++w) {
                CK(hipEventRecord(e0));
                if (w == 0) hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, 0, a, n, sink);
                if (w == 1) hipLaunchKernelGGL(write_kernel, dim3(grid), dim3(256), 0, 0, b, n);
                if (w == 2) hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, 0, a, b, n);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep && ms < best[w]) best[w] = ms;  // rep 0 warms up
            }
        }
        std::printf("grid %5d: read %.0f GB/s  write %.0f GB/s  copy %.0f GB/s (read+write bytes)\n", grid,
                    bytes / best[0] / 1e6, bytes / best[1] / 1e6, 2 * bytes / best[2] / 1e6);
    }
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(sink));
    return 0;
}
