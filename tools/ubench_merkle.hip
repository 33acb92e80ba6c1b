// ubench_merkle.hip -- diagnostic (not product code): times nb_merkle_device on
// C2's shape (10M x 16-byte records) for a build of merkle_kernels.hip with the
// level-kernel geometry given by -DNB_MERKLE_THREADS / -DNB_MERKLE_SUBLEVELS.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../nasp-key-value-engine_amd/csrc/merkle_kernels.hip"

int nb_internal_fail(int code, const char *msg) {
    std::printf("error %d: %s\n", code, msg);
    return code;
}

__global__ void k_fill(uint64_t *p, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        uint64_t x = i + 0x9E3779B97F4A7C15ull;
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        p[i] = x ^ (x >> 27);
    }
}

int main() {
    const uint64_t n = 10000000;
    uint8_t *data;
    uint64_t *tree;
    (void)hipMalloc(&data, n * 16 + 64);
    (void)hipMalloc(&tree, nb_merkle_tree_size(n) * 8);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(data), 2 * n);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
        (void)hipEventRecord(a);
        nb_merkle_device(data, nullptr, 16, n, 0, tree, nullptr);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (r && ms < best) best = ms;
    }
    uint64_t root;
    (void)hipMemcpy(&root, tree + nb_merkle_tree_size(n) - 1, 8, hipMemcpyDeviceToHost);
    std::printf("threads %d sublevels %d: %.4f ms  root %llu\n", NB_MERKLE_THREADS, NB_MERKLE_SUBLEVELS,
                best, (unsigned long long)root);
    return 0;
}
